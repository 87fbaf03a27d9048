"""Study (host only): would longest-first scheduling or per-item stage fusion
shorten the ObjPose queues? Uses the host build of mk_rpp.h on the bench
scene's first-ObjPose problems (tools/rpp_iter_hist.py's frames).

1. Lane-level list scheduling of the first-ObjPose jobs at the bench's jobs
   per lane: FIFO (the queue order) against a probe round of K AbsKernel
   trips for every job, then the unfinished ones longest-first by the
   predicted remaining count (the |de/e| convergence rate over the last 8
   trips, as mk_rpp.h op_predict), and against the exact-length LPT bound.
2. Per rig, (longest first ObjPose + longest candidate ObjPose) against the
   longest (first + candidate) chain of one item: what running an item's
   candidate ObjPoses as soon as its first one ends could save in latency.

    python tools/objpose_sched_sim.py [rigs]
"""
import ctypes as C
import heapq
import os
import sys
from concurrent.futures import ThreadPoolExecutor

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import _hostcheck as HC  # noqa: E402
import _oracle as O  # noqa: E402
from mantis_amd import synth  # noqa: E402

TOL = 1e-5  # RPP.cpp ObjPose stop test
W, H = 1280, 720


def problems(n_rigs):
    K, D = synth.intrinsics(W, H)
    white, red, green = synth.load_map()
    rng = np.random.default_rng(1000)
    ext = synth.rig_extrinsics(4)
    cams = []
    for r in range(n_rigs):
        Twb = synth.random_base_pose(rng)
        for c in range(4):
            Twc = Twb @ ext[c]
            cams.append((r * 4 + c, synth.make_cam(Twc[:3, :3], Twc[:3, 3], W, H)))

    def one(j):
        i, cam = j
        d = O.Oracle(white, red, green, seed=1).process(synth.render_host(cam, synth.frame_seed(3, i)), K, D)
        tp = np.array(d.test_pts)[: d.n_quads].reshape(d.n_quads, 4, 2)
        out, h = [], 0.16
        for q in range(d.n_quads):
            ip = np.ascontiguousarray(np.vstack([tp[q].T, np.ones(4)]))
            for o in range(2):
                sy = [h, h, -h, -h] if o == 0 else [-h, -h, h, h]
                model = np.ascontiguousarray(np.array([[h, -h, -h, h], sy, [0, 0, 0, 0.0]]))
                it = np.zeros(6, np.int32)
                HC.lib().hc_rpp_iters(model.ctypes.data_as(C.POINTER(C.c_double)),
                                      ip.ctypes.data_as(C.POINTER(C.c_double)), it.ctypes.data_as(C.POINTER(C.c_int32)))
                out.append((i // 4, o, it.copy(), model, ip))
        return out

    with ThreadPoolExecutor(8) as ex:
        return [x for r in ex.map(one, cams) for x in r]


def traces(res):
    L = HC.lib()
    L.hc_objpose_trace.restype = C.c_int
    its, E = [], []
    for _, o, _, m, ip in res:
        if o:
            continue  # orientation 1 mirrors orientation 0 (same chain)
        e = np.zeros(4000)
        ipc = ip.copy()
        n = L.hc_objpose_trace(m.ctypes.data_as(C.POINTER(C.c_double)), ipc.ctypes.data_as(C.POINTER(C.c_double)),
                               None, 4000, e.ctypes.data_as(C.POINTER(C.c_double)))
        its.append(n)
        E.append(e)
    return np.array(its), np.array(E)


def predict(e, it, K, span=8):
    if it <= K:
        return it
    r1 = abs((e[K - 2] - e[K - 1]) / e[K - 2])
    r0 = abs((e[K - 2 - span] - e[K - 1 - span]) / e[K - 2 - span])
    if not r1 > TOL:
        return K + 1
    rho = (r1 / r0) ** (1 / span) if (r0 > 0 and r1 < r0) else 1.0
    if not rho < 0.99999:
        return 1e6
    return K + max(0.0, np.log(TOL / r1) / np.log(rho)) + 1


def lanes_makespan(durs, lanes):
    h = [0.0] * lanes
    for d in durs:
        heapq.heappush(h, heapq.heappop(h) + d)
    return max(h)


def main():
    res = problems(int(sys.argv[1]) if len(sys.argv) > 1 else 8)
    its, E = traces(res)
    n = len(its)
    rng = np.random.default_rng(0)
    print(f"{n} first-ObjPose chains: mean {its.mean():.1f} max {its.max()} iterations")
    for lanes in (n // 38, n // 19, n // 10):
        fifo = lanes_makespan(its[rng.permutation(n)], lanes)
        lpt = lanes_makespan(np.sort(its)[::-1], lanes)
        row = [f"lanes {lanes}: FIFO {fifo:.0f}, LPT bound {lpt:.0f}"]
        for K in (16, 24, 32, 48):
            t0 = lanes_makespan(np.minimum(its[rng.permutation(n)], K), lanes)
            rem = np.flatnonzero(its > K)
            p = np.array([predict(E[j], its[j], K) for j in rem])
            t1 = lanes_makespan(its[rem[np.argsort(-p)]] - K, lanes)
            cc = np.corrcoef(np.log(p), np.log(its[rem]))[0, 1]
            row.append(f"probe {K}: {t0 + t1:.0f} (log-corr {cc:.2f})")
        print("; ".join(row))
    by = {}
    for rig, _, it, _, _ in res:
        by.setdefault(rig, []).append(it)
    staged, fused = [], []
    for items in by.values():
        cand = [max([v for v in i[1:] if v >= 0] or [0]) for i in items]
        staged.append(max(i[0] for i in items) + max(cand))
        fused.append(max(i[0] + c for i, c in zip(items, cand)))
    staged, fused = np.array(staged), np.array(fused)
    print(f"per rig: staged {np.median(staged):.0f} vs per-item fused {np.median(fused):.0f} iterations "
          f"(median saving {np.median((staged - fused) / staged) * 100:.1f} %)")


if __name__ == "__main__":
    main()
