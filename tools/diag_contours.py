"""Diagnostics: per-phase ticks of k_frame_contours over a config-3 batch."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np

import mantis_amd as M
from mantis_amd import synth

W, H = 1280, 720
rigs = int(sys.argv[1]) if len(sys.argv) > 1 else 32
white, red, green = synth.load_map()
K, D = synth.intrinsics(W, H)
n = rigs * 4
m = M.Mantis(M.default_config(max_cams=n, max_width=W, max_height=H))
m.set_map(white, red, green)
rng = np.random.default_rng(1000)
ext = synth.rig_extrinsics(4)
cams, Tbc = [], []
for r in range(rigs):
    Twb = synth.random_base_pose(rng)
    for c in range(4):
        Twc = Twb @ ext[c]
        cams.append(synth.make_cam(Twc[:3, :3], Twc[:3, 3], W, H))
        Tbc.append(ext[c])
fb = W * H * 3
dev = m.device_alloc(n * fb)
m.synth_render(cams, [synth.frame_seed(3, i) for i in range(n)], dev)
imgs = [M.make_image(None, K, D, T_base_cam=Tbc[i], device_ptr=dev + i * fb, width=W, height=H) for i in range(n)]
m.process(imgs, rigs=rigs)
m.set_profiling(True)
m.process(imgs, rigs=rigs)
print("stages", [(k, round(v, 3)) for k, v in m.stage_times()], flush=True)
C = np.array([m.frame_counters(i) for i in range(n)])
names = ["borders", "points", "raw_q", "quads", "gen", "hyps", "pf", "goff", "ovf", "cand"]
print("longest walk steps mean", C[:, 18].mean(), "max", C[:, 18].max())
for j, nm in enumerate(names):
    print(f"{nm:8s} mean {C[:, j].mean():10.1f} max {C[:, j].max()}")
T = C[:, 10:16].astype(float) * 0.01  # us
ph = ["scan", "compact", "approx_short", "approx_long", "dedup", "rest"]
prev = np.zeros(n)
for j, nm in enumerate(ph):
    d = T[:, j] - prev
    print(f"{nm:8s} us mean {d.mean():9.1f} max {d.max():9.1f}")
    prev = T[:, j]
