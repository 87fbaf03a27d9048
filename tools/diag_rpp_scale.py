"""Diagnostics: RPP batch time vs problem count (realistic 4-corner problems)."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np

import mantis_amd as M
from mantis_amd import synth

m = M.Mantis(max_cams=4)
rng = np.random.default_rng(5)
s = 0.16
sq = [np.array([[s, -s, -s, s], [s, s, -s, -s], [0, 0, 0, 0.0]]), np.array([[s, -s, -s, s], [-s, -s, s, s], [0, 0, 0, 0.0]])]
N = 1 << 17
ips, ops = np.zeros((N, 4, 2)), np.zeros((N, 4, 3))
for k in range(N):
    R = synth.rot_z(rng.uniform(0, 6.3)) @ synth.NADIR @ synth.rot_x(rng.normal() * 0.3)
    t = np.array([rng.normal() * 0.3, rng.normal() * 0.3, rng.uniform(0.8, 3)])
    mm = sq[k % 2]
    Q = R.T @ mm + t[:, None]
    ips[k] = (np.vstack([Q[0] / Q[2], Q[1] / Q[2]]) + rng.normal(size=(2, 4)) * 0.003).T
    ops[k] = mm.T
sizes = [int(a) for a in sys.argv[1:]] or [64, 1024, 4096, 16384, 65536, 131072]
for n in sizes:
    m.rpp(ips[:n], ops[:n])
    t0 = time.perf_counter()
    m.rpp(ips[:n], ops[:n])
    dt = time.perf_counter() - t0
    print(f"n={n:7d} {dt*1e3:9.2f} ms  {dt/n*1e6:8.3f} us/problem", flush=True)
