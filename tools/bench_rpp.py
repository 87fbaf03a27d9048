"""RPP microbenchmark (GPU box): the (quad, orientation) problems of synthetic
config-3 frames, detected by the library itself, solved by mantis_rpp_batch at
several batch sizes; prints per-phase event times. A/B builds via
MANTIS_AMD_LIB=<path>. Diagnostic tool only."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np

import mantis_amd as M
from mantis_amd import synth

W, H = 1280, 720


def problems(n_frames=64):
    white, red, green = synth.load_map()
    K, D = synth.intrinsics(W, H)
    m = M.Mantis(M.default_config(max_cams=n_frames, max_width=W, max_height=H))
    m.set_map(white, red, green)
    rng = np.random.default_rng(1000)
    ext = synth.rig_extrinsics(4)
    cams = []
    for r in range(n_frames // 4):
        Twb = synth.random_base_pose(rng)
        for c in range(4):
            Twc = Twb @ ext[c]
            cams.append(synth.make_cam(Twc[:3, :3], Twc[:3, 3], W, H))
    fb = W * H * 3
    dev = m.device_alloc(n_frames * fb)
    m.synth_render(cams, [synth.frame_seed(3, i) for i in range(n_frames)], dev)
    m.synchronize()
    imgs = [M.make_image(None, K, D, device_ptr=dev + i * fb, width=W, height=H) for i in range(n_frames)]
    m.process(imgs, n_frames // 4)
    s = 0.16
    mods = [np.array([[s, s, 0], [-s, s, 0], [-s, -s, 0], [s, -s, 0.0]]),
            np.array([[s, -s, 0], [-s, -s, 0], [-s, s, 0], [s, s, 0.0]])]
    ip, op = [], []
    for i in range(n_frames):
        d = m.frame_debug(i)
        for q in range(d.n_quads):
            tp = np.array(d.test_pts[q][:]).reshape(4, 2)
            for o in range(2):
                ip.append(tp)
                op.append(mods[o])
    return m, np.array(ip), np.array(op)


def main():
    m, ip, op = problems()
    out = {"lib": os.path.basename(M.LIB_PATH), "base_problems": len(ip)}
    for n in [int(a) for a in (sys.argv[1:] or ["600", "38400", "153600"])]:
        reps = (n + len(ip) - 1) // len(ip)
        I = np.concatenate([ip] * reps)[:n]
        O = np.concatenate([op] * reps)[:n]
        m.set_profiling(True)
        m.rpp(I, O)
        best = None
        for _ in range(3):
            R, t, e, st = m.rpp(I, O)
            kt = dict(m.stage_times())
            tot = sum(kt.values())
            if best is None or tot < best[0]:
                best = (tot, kt)
        m.set_profiling(False)
        out[str(n)] = {k: round(v, 3) for k, v in best[1].items()}
        out[str(n)]["total_ms"] = round(best[0], 3)
        out[str(n)]["checksum"] = float(np.sum(e[:, 0]))
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
