"""N>1 paths on CPU with torch.distributed over gloo (world size 2).

* Rig GN sharded by camera: each rank accumulates its cameras' 28 doubles
  with the library's own residual rows (mk_gn.h, host build through
  tests/_hostcheck.py), the all-reduce sums them, every rank solves the same
  6x6 system with the library's mantis_gn_solve — the final pose is identical
  on both ranks, equal to the single-process result, and the accumulators
  agree with the numpy restatement (tests/_gn_ref.py).
* bench.py's weak-scaling reduction: the MAX of the per-rank times is used.
* Config 5's argmin exchange: the library's mantis_argmin_pick over the
  all-gathered (err, index) pairs.
* Camera-sharded rigs (mantis_process_rig_sharded) at world 2, 3 (8 cameras
  over 3 ranks: 3 / 3 / 2, padding slots) and 4: the library's own
  cross-rank bookkeeping (mk_shard.h, host build) -- PF-flag pairs ->
  all-gather -> per-frame cv::RNG offsets; camera records -> all-gather ->
  merge -> rig fusion and rng_state_after -- on the per-frame flags and camera
  records of a real one-GPU batch (tests/golden/shard_batch.npz, written by
  tests/golden/make_shard_fixture.py on the GPU box): every rank's offsets
  equal the sequential prefix, and its fused rig results equal the batch's,
  byte for byte.
* bench.py --gpus 2 without torchrun spawns two ranks of itself, which get as
  far as creating the library context (no GPU here) and fail with a clear
  message.
"""
import os
import socket

import numpy as np
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import _gn_ref as G
import _hostcheck as HC


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _scene():
    rng = np.random.default_rng(12)
    T_true = G.exp_se3_right(np.eye(4), np.array([0.2, -0.1, 1.4, 0.05, -0.03, 0.7]))
    ext = []
    for c in range(4):
        E = np.eye(4)
        ang = c * np.pi / 2
        E[:3, :3] = np.array([[np.cos(ang), -np.sin(ang), 0], [np.sin(ang), np.cos(ang), 0], [0, 0, 1]])
        E[:3, 3] = [0.1 * np.cos(ang), 0.1 * np.sin(ang), 0]
        ext.append(E)
    obs = G.synth_rig_obs(rng, T_true, ext, n_per_cam=30, noise=5e-4)
    T0 = G.exp_se3_right(T_true, np.array([0.03, -0.02, 0.04, 0.02, -0.015, 0.03]))
    return T_true, T0, ext, obs


def _worker(rank, world, port, out):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from mantis_amd import rig

    T_true, T0, ext, obs = _scene()
    mine = rig.shard_cameras(len(ext), rank, world)
    local = obs[np.isin(obs[:, 0].astype(int), mine)]

    def accumulate(T):
        return HC.gn_accumulate(T, ext, local) if len(local) else np.zeros(28)

    def allreduce(acc):
        t = torch.from_numpy(acc)
        dist.all_reduce(t, op=dist.ReduceOp.SUM)

    T, costs = rig.gn_refine(T0, accumulate, allreduce, iterations=6)
    # bench.py timing reduction: max over ranks
    t = torch.tensor([1.0 + rank], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    out[rank] = (T, costs, float(t.item()), mine)
    dist.destroy_process_group()


def test_camera_sharded_gn_world2():
    from mantis_amd import rig

    world = 2
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_worker, args=(world, _free_port(), out), nprocs=world, join=True)
    T_true, T0, ext, obs = _scene()
    T1, costs1 = rig.gn_refine(T0, lambda T: HC.gn_accumulate(T, ext, obs), None, iterations=6)
    np.testing.assert_allclose(HC.gn_accumulate(T0, ext, obs), G.gn_accumulate(T0, ext, obs), rtol=1e-12,
                               atol=1e-15)
    Ta, ca, ma, sa = out[0]
    Tb, cb, mb, sb = out[1]
    assert sa == [0, 2] and sb == [1, 3]
    assert ma == mb == 2.0
    assert np.array_equal(Ta, Tb)  # identical solve on every rank
    np.testing.assert_allclose(Ta, T1, rtol=0, atol=1e-12)
    np.testing.assert_allclose(ca, costs1, rtol=1e-9)
    assert costs1[-1] < 1e-3 * costs1[0]
    np.testing.assert_allclose(Ta[:3, 3], T_true[:3, 3], atol=2e-3)


def _argmin_worker(rank, world, port, out):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import mantis_amd as M
    from mantis_amd import dense

    err = _dense_errors()
    lo, hi = dense.shard_range(len(err), rank, world)
    local = err[lo:hi]
    # device-side rule per shard (k_argmin): first minimum of the block
    pair = torch.tensor([local.min(), lo + int(np.argmin(local))] if len(local) else [np.finfo(np.float64).max, -1.0],
                        dtype=torch.float64)
    pairs = [torch.zeros(2, dtype=torch.float64) for _ in range(world)]
    dist.all_gather(pairs, pair)  # the ncclAllGather of mantis_score_argmin, 16 B per rank
    out[rank] = M.argmin_pick(torch.stack(pairs).numpy())
    dist.destroy_process_group()


def _dense_errors():
    rng = np.random.default_rng(5)
    err = rng.integers(1000, 5000, 16200).astype(np.float64) / 7.0
    m = err.min()
    err[[9000, 8100, 12000]] = m - 1.0  # ties on both sides of the 2-rank boundary (8100)
    return err


def test_hypothesis_sharded_argmin_world2():
    """Config 5: 16,200 hypotheses split over ranks; the exchanged (err, index)
    pairs give every rank the global first minimum."""
    world = 2
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_argmin_worker, args=(world, _free_port(), out), nprocs=world, join=True)
    err = _dense_errors()
    want = (float(err.min()), int(np.argmin(err)))
    assert want[1] == 8100
    assert out[0] == want and out[1] == want


def test_argmin_pick_rules():
    import mantis_amd as M
    from mantis_amd import dense

    big = np.finfo(np.float64).max
    assert M.argmin_pick([[3.0, 7], [3.0, 2], [4.0, 0]]) == (3.0, 2)
    assert M.argmin_pick([[big, -1], [5.0, 11]]) == (5.0, 11)
    assert M.argmin_pick([[big, -1], [big, -1]])[1] == -1
    assert M.argmin_pick([[big, 4], [big, 9]]) == (big, 4)  # every hypothesis unprojectable: first index
    spans = [dense.shard_range(16200, r, 8) for r in range(8)]
    assert spans[0] == (0, 2025) and spans[-1] == (14175, 16200)
    assert all(spans[i][1] == spans[i + 1][0] for i in range(7))
    assert dense.shard_range(5, 3, 4) == (4, 5) and dense.shard_range(2, 3, 4) == (2, 2)


SHARD_FIXTURE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "shard_batch.npz")


def _shard_worker(rank, world, port, out):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from mantis_amd import rig

    z = np.load(SHARD_FIXTURE)
    R, Cn, per = int(z["rigs"]), int(z["cams"]), int(z["per"])
    ng = R * Cn
    cams = rig.shard_cameras(Cn, rank, world)
    gidx = HC.shard_global_indices(R, cams, Cn)
    assert list(gidx) == [r * Cn + c for r in range(R) for c in cams]
    nl_max = -(-Cn // world)
    slots = R * nl_max
    # (global index, PF flag) pairs -> all-gather (the library's ncclAllGather) -> offsets
    pairs = torch.from_numpy(HC.shard_pack_pairs(gidx, z["pf"][gidx], slots))
    got = [torch.zeros_like(pairs) for _ in range(world)]
    dist.all_gather(got, pairs)
    flags, off, tot = HC.shard_offsets(torch.cat(got).numpy(), ng, per)
    # camera records -> all-gather -> merge -> fusion + rng_state_after
    recs = torch.from_numpy(HC.shard_make_recs(z["cam_bytes"][gidx], z["tbc"][gidx], gidx, slots))
    rgot = [torch.zeros_like(recs) for _ in range(world)]
    dist.all_gather(rgot, recs)
    code, allb, tall = HC.shard_merge(torch.cat(rgot).numpy(), ng)
    rigs = HC.rig_results(R, Cn, allb, tall, flags, z["states"])
    out[rank] = (cams, flags, off[gidx], off, tot, code, allb, tall, rigs, slots - len(gidx))
    dist.destroy_process_group()


def _check_shard_world(world):
    z = np.load(SHARD_FIXTURE)
    cs, rsz, _ = HC.sizes()
    assert int(z["cam_result_size"]) == cs and int(z["result_size"]) == rsz, "fixture layout differs from mantis.h"
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_shard_worker, args=(world, _free_port(), out), nprocs=world, join=True)
    pf, per = z["pf"], int(z["per"])
    seq = per * np.concatenate([[0], np.cumsum(pf)[:-1]])  # sequential offsets, global frame order
    assert 0 < pf.sum() < len(pf)
    owners = []
    for r in range(world):
        cams, flags, off_local, off_all, tot, code, allb, tall, rigs, pad = out[r]
        owners += cams
        assert code == 0
        assert np.array_equal(flags, pf)
        assert np.array_equal(off_all, seq) and tot == per * pf.sum()
        gidx = HC.shard_global_indices(int(z["rigs"]), cams, int(z["cams"]))
        assert np.array_equal(off_local, seq[gidx])
        assert np.array_equal(allb, z["cam_bytes"]) and np.array_equal(tall, z["tbc"].reshape(-1, 16))
        assert np.array_equal(rigs, z["rig_bytes"]), f"rank {r}: fused rig results differ from the batch's"
    assert sorted(owners) == list(range(int(z["cams"])))
    return out


def test_sharded_bookkeeping_world2():
    _check_shard_world(2)


def test_sharded_bookkeeping_world3_uneven():
    out = _check_shard_world(3)
    assert [len(out[r][0]) for r in range(3)] == [3, 3, 2]  # 8 cameras: rank 2 sends padding slots
    assert out[0][9] == 0 and out[2][9] == 3  # rank 2: one padding slot per rig


def test_sharded_bookkeeping_world4():
    _check_shard_world(4)


def test_shard_merge_rejects_bad_ownership():
    """A camera sent by two ranks, or by none, is an error (the library
    returns MANTIS_ERR_ARG with a message instead of fusing)."""
    z = np.load(SHARD_FIXTURE)
    R, Cn = int(z["rigs"]), int(z["cams"])
    ng = R * Cn
    g = np.arange(ng, dtype=np.int32)
    recs = HC.shard_make_recs(z["cam_bytes"], z["tbc"], g, ng)
    rs = HC.sizes()[2]
    code, allb, _ = HC.shard_merge(recs, ng)
    assert code == 0 and np.array_equal(allb, z["cam_bytes"])
    dup = np.concatenate([recs, recs[:rs]])
    assert HC.shard_merge(dup, ng)[0] == 1
    assert HC.shard_merge(recs[: (ng - 1) * rs], ng)[0] == 2
    g2 = g.copy()
    g2[3] = ng + 5
    assert HC.shard_merge(HC.shard_make_recs(z["cam_bytes"], z["tbc"], g2, ng), ng)[0] == 3


def test_bench_launcher_spawns_ranks():
    """`bench.py --gpus 2` (no torchrun): the launcher never touches the GPU,
    starts 2 ranks that rendezvous over gloo and stop at context creation."""
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK")}
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "2", "--no-cpu"], env=env,
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 1
    for k in range(2):
        assert f"bench rank {k}/2: cannot create a library context on device {k}" in r.stderr, r.stderr
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "2"],
                       env=dict(env, WORLD_SIZE="1"), capture_output=True, text=True, timeout=120)
    assert r.returncode == 2 and "WORLD_SIZE=1" in r.stderr
