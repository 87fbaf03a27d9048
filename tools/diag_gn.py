"""Diagnostics: rig pose error vs synthetic truth with and without cfg.gn_enable."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np

import mantis_amd as M
from mantis_amd import synth


def qmat(q):
    x, y, z, w = q
    return np.array([[1 - 2 * (y * y + z * z), 2 * (x * y - z * w), 2 * (x * z + y * w)],
                     [2 * (x * y + z * w), 1 - 2 * (x * x + z * z), 2 * (y * z - x * w)],
                     [2 * (x * z - y * w), 2 * (y * z + x * w), 1 - 2 * (x * x + y * y)]])


n = int(sys.argv[1]) if len(sys.argv) > 1 else 16
K, D = synth.intrinsics()
ext = synth.rig_extrinsics(4)
rng = np.random.default_rng(21)
imgs, truth = [], []
for r in range(n):
    Twb = synth.random_base_pose(rng)
    truth.append(Twb)
    for c in range(4):
        Twc = Twb @ ext[c]
        fr = synth.render_host(synth.make_cam(Twc[:3, :3], Twc[:3, 3]), synth.frame_seed(7, 10 * r + c))
        imgs.append(M.make_image(fr, K, D, T_base_cam=ext[c]))
res = {}
for gn in (0, 1):
    m = M.Mantis(M.default_config(max_cams=4 * n, max_width=1280, max_height=720, gn_enable=gn, gn_iterations=8))
    m.set_map(*synth.load_map())
    res[gn] = m.process(imgs, rigs=n)[0]
    m.close()
for r in range(n):
    out = []
    for gn in (0, 1):
        R = res[gn][r]
        p = np.array(R.position)
        ang = np.degrees(np.arccos(np.clip((np.trace(qmat(R.orientation_xyzw).T @ truth[r][:3, :3]) - 1) / 2, -1, 1)))
        out.append(f"pos {np.linalg.norm(p - truth[r][:3, 3]):.4f} ang {ang:.3f}")
    print(r, res[0][r].publish, " | ".join(out), "it", res[1][r].gn_iterations, "cost", f"{res[1][r].gn_cost:.3e}")
