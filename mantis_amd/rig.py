"""Rig Gauss-Newton refinement across camera shards (e).

Each rank owns the cameras c with c % world == rank. Per iteration it forms
its cameras' 28 accumulators (upper-triangle J^T J, J^T r, r^T r) about the
shared base pose, the ranks sum them (RCCL all-reduce of 28 doubles through
mantis_gn_allreduce, or any `allreduce` callable, e.g. torch.distributed over
gloo in tests), and every rank solves the same 6x6 system with
mantis_gn_solve — no broadcast needed, all ranks hold identical poses.
"""
import ctypes as C

import numpy as np

from . import lib


def shard_cameras(n_cams, rank, world):
    return [c for c in range(n_cams) if c % world == rank]


def gn_refine(T_w_b, accumulate, allreduce=None, iterations=5, lam=1e-9):
    """accumulate(T) -> 28 local doubles; allreduce(np.ndarray) sums in place
    across ranks (None for one rank). Returns (T_w_b, per-iteration cost)."""
    T = np.ascontiguousarray(T_w_b, np.float64).copy()
    costs = []
    for _ in range(iterations):
        acc = np.ascontiguousarray(accumulate(T), np.float64)
        if allreduce is not None:
            allreduce(acc)
        costs.append(float(acc[27]))
        st = lib().mantis_gn_solve(acc.ctypes.data_as(C.c_void_p), C.c_double(lam), T.ctypes.data_as(C.c_void_p),
                                   None)
        if st != 0:
            break
    return T, costs
