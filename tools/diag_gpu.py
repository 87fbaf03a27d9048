"""GPU diagnostics: run each stage with timing, printing progress as it goes."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import numpy as np

import _oracle as O
import mantis_amd as M
from mantis_amd import synth


def log(*a):
    print(*a, flush=True)


which = sys.argv[1] if len(sys.argv) > 1 else "all"
white, red, green = synth.load_map()
K, D = synth.intrinsics()
m = M.Mantis(max_cams=8)
m.set_map(white, red, green)
log("ctx ok")
if which in ("rpp", "all"):
    s = 0.16
    sq = np.array([[s, -s, -s, s], [s, s, -s, -s], [0, 0, 0, 0.0]])
    for n in (1, 4, 64, 256):
        rng = np.random.default_rng(n)
        ips, ops = [], []
        for k in range(n):
            R = synth.rot_z(rng.uniform(0, 6.28)) @ synth.NADIR @ synth.rot_x(rng.normal() * 0.3)
            t = np.array([rng.normal() * 0.3, rng.normal() * 0.3, rng.uniform(0.8, 3)])
            Q = R.T @ sq + t[:, None]
            ips.append(np.vstack([Q[0] / Q[2], Q[1] / Q[2]]).T.copy())
            ops.append(sq.T.copy())
        t0 = time.time()
        R, t, e, st = m.rpp(np.array(ips), np.array(ops))
        log(f"rpp n={n} {time.time()-t0:.3f}s status={st[:4]} err0={e[0]}")
        ref = O.rpp(sq, np.vstack([ips[0].T, np.ones(4)]))
        log("  oracle", ref[0], np.abs(ref[1] - R[0]).max(), ref[3][:2])
if which in ("score", "all"):
    rng = np.random.default_rng(3)
    R, pos = synth.random_pose(rng)
    img = synth.render_host(synth.make_cam(R, pos), 5)
    c2w = np.array([synth.truth_c2w(R, pos)] * 8)
    for fast in (1, 0):
        t0 = time.time()
        e, n = m.score(M.make_image(img, K, D), c2w, fast=bool(fast))
        log(f"score fast={fast} {time.time()-t0:.3f}s", e[:2], n[:2])
        orc = O.Oracle(white, red, green)
        log("  oracle", orc.score(img, K, D, c2w[:2], fast=bool(fast)))
if which in ("full", "all"):
    rng = np.random.default_rng(1234)
    imgs = []
    for f in range(2):
        R, pos = synth.random_pose(rng)
        imgs.append(synth.render_host(synth.make_cam(R, pos), synth.frame_seed(2, f)))
    m.set_profiling(True)
    t0 = time.time()
    rig, cams = m.process([M.make_image(i, K, D) for i in imgs], rigs=2)
    log(f"full {time.time()-t0:.3f}s", [(c.reason, c.n_quads, c.n_hyps, c.pf_error) for c in cams])
    log(m.kernel_times())
log("done")
