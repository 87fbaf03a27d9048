"""Diagnostic: ObjPose iteration counts per RPP job on the bench scene
(host build of mk_rpp.h via tests/_hostcheck.py; quads/test points from the
oracle). Prints the distribution of first-ObjPose and candidate iterations
and the longest jobs, i.e. the serial tail of the persistent queues, and
writes the 16 longest first-ObjPose problems to tools/objpose_long.bin."""
import os
import sys
from concurrent.futures import ThreadPoolExecutor

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import ctypes as C

import numpy as np

import _hostcheck as HC
import _oracle as O
from mantis_amd import synth

n_rigs = int(sys.argv[1]) if len(sys.argv) > 1 else 32
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
    fr = synth.render_host(cam, synth.frame_seed(3, i))
    orc = O.Oracle(white, red, green, seed=1)
    d = orc.process(fr, K, D)
    n = d.n_quads
    tp = np.array(d.test_pts)[:n].reshape(n, 4, 2)
    out = []
    h = 0.16
    for q in range(n):
        ip = np.vstack([tp[q].T, np.ones(4)])
        for o in range(2):
            sy = [h, h, -h, -h] if o == 0 else [-h, -h, h, h]
            model = np.array([[h, -h, -h, h], sy, [0, 0, 0, 0.0]])
            it = np.zeros(6, np.int32)
            HC.lib().hc_rpp_iters(model.ctypes.data_as(C.POINTER(C.c_double)),
                                  np.ascontiguousarray(ip).ctypes.data_as(C.POINTER(C.c_double)),
                                  it.ctypes.data_as(C.POINTER(C.c_int32)))
            out.append((i, q, o, it.copy(), np.concatenate([model.ravel(), ip.ravel()])))
    return out


with ThreadPoolExecutor(8) as ex:
    res = [x for r in ex.map(one, jobs) for x in r]
first = np.array([x[3][0] for x in res])
cand = np.array([v for x in res for v in x[3][1:] if v >= 0])
print(f"{len(jobs)} frames, {len(first)} first-ObjPose jobs, {len(cand)} candidate jobs")
for name, a in (("first", first), ("cand", cand)):
    print(name, "sum", a.sum(), "mean", round(a.mean(), 1), "p50", np.percentile(a, 50), "p99", np.percentile(a, 99),
          "max", a.max(), "top", np.sort(a)[-8:])
worst = sorted(res, key=lambda x: -x[3].max())[:8]
for w in worst:
    print("frame", w[0], "quad", w[1], "orient", w[2], "iters", list(w[3]))
# the longest first-ObjPose problems (model 3x4 then image points 3x4, row-major
# float64) for tools/objpose_lat.hip
longest = sorted(res, key=lambda x: -x[3][0])[:16]
np.stack([x[4] for x in longest]).astype(np.float64).tofile(os.path.join(ROOT, "tools", "objpose_long.bin"))
