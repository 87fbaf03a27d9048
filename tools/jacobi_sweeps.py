"""Writes the RPP problems of the bench scene (quads from the oracle, both
model orientations) for tools/jacobi_sweeps.cpp and runs it.
Usage: jacobi_sweeps.py [rigs]"""
import os
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests")]
import numpy as np

import _oracle as O
from mantis_amd import synth

n_rigs = int(sys.argv[1]) if len(sys.argv) > 1 else 8
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
    d = O.Oracle(white, red, green, seed=1).process(fr, K, D)
    n = d.n_quads
    tp = np.array(d.test_pts)[:n].reshape(n, 4, 2)
    h = 0.16
    out = []
    for q in range(n):
        ip = np.vstack([tp[q].T, np.ones(4)])
        for sy in ([h, h, -h, -h], [-h, -h, h, h]):
            out.append(np.concatenate([np.array([[h, -h, -h, h], sy, [0, 0, 0, 0.0]]).ravel(), ip.ravel()]))
    return out


with ThreadPoolExecutor(8) as ex:
    probs = [x for r in ex.map(one, jobs) for x in r]
os.makedirs(os.path.join(ROOT, "build"), exist_ok=True)
pb = os.path.join(ROOT, "build", "objpose_problems.bin")
np.stack(probs).astype(np.float64).tofile(pb)
exe = os.path.join(ROOT, "build", "jacobi_sweeps")
subprocess.check_call(["g++", "-O2", "-std=c++17", "-ffp-contract=off", "-o", exe,
                       os.path.join(ROOT, "tools", "jacobi_sweeps.cpp")])
print(len(probs), "problems")
subprocess.check_call([exe, pb])
