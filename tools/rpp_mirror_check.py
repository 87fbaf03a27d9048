"""Check (host build of mk_rpp.h) that the first ObjPose of the two model
orientations of a quad are mirror images: R1 = R0 diag(1, -1, -1), t, both
errors, the iteration count and the rewritten image points identical, bit
for bit -- the property k_objpose_q<0> / op_end<0> use to run one ObjPose per
quad. Usage: rpp_mirror_check.py [rigs] (bench scene, quads from the oracle)."""
import ctypes as C
import os
import sys
from concurrent.futures import ThreadPoolExecutor

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests")]
import numpy as np

import _hostcheck as HC
import _oracle as O
from mantis_amd import synth


def first_objpose(model, iprts):
    L = HC.lib()
    P = lambda a: a.ctypes.data_as(C.c_void_p)
    R, t, e, it, Q = np.zeros(9), np.zeros(3), np.zeros(2), np.zeros(1, np.int32), np.zeros(12)
    L.hc_first_objpose(P(np.ascontiguousarray(model)), P(np.ascontiguousarray(iprts)), P(R), P(t), P(e), P(it), P(Q))
    return R.reshape(3, 3), t, e, int(it[0]), Q


def mirror_pair_ok(ip, h=0.16):
    """ip: 3 x 4 homogeneous normalized image points of one quad."""
    models = [np.array([[h, -h, -h, h], sy, [0, 0, 0, 0.0]]) for sy in ([h, h, -h, -h], [-h, -h, h, h])]
    a, b = (first_objpose(m, ip) for m in models)
    S = np.diag([1.0, -1.0, -1.0])
    return (np.array_equal(b[0], a[0] @ S) and np.array_equal(a[1], b[1]) and np.array_equal(a[2], b[2])
            and a[3] == b[3] and np.array_equal(a[4], b[4]))


def frame_quads(n_rigs):
    W, H = 1280, 720
    K, D = synth.intrinsics(W, H)
    white, red, green = synth.load_map()
    rng = np.random.default_rng(1000)
    ext = synth.rig_extrinsics(4)
    jobs = []
    for r in range(n_rigs):
        Twb = synth.random_base_pose(rng)
        for c in range(4):
            Twc = Twb @ ext[c]
            jobs.append((r * 4 + c, synth.make_cam(Twc[:3, :3], Twc[:3, 3], W, H)))

    def one(j):
        i, cam = j
        d = O.Oracle(white, red, green, seed=1).process(synth.render_host(cam, synth.frame_seed(3, i)), K, D)
        tp = np.array(d.test_pts)[: d.n_quads].reshape(-1, 4, 2)
        return [np.vstack([q.T, np.ones(4)]) for q in tp]

    with ThreadPoolExecutor(8) as ex:
        return [q for f in ex.map(one, jobs) for q in f]


if __name__ == "__main__":
    quads = frame_quads(int(sys.argv[1]) if len(sys.argv) > 1 else 16)
    ok = sum(mirror_pair_ok(q) for q in quads)
    print(f"{len(quads)} quads: exact mirror relation {ok}")
    sys.exit(0 if ok == len(quads) else 1)
