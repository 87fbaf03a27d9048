"""Phase times of k_score_final per frame (a library built with
-DMK_SCORE_TICKS, MANTIS_AMD_LIB): one context, one batch of bench rigs;
median / p90 of each phase over the frames that reach the particle filter.
Phases: shift tasks, unsure drain, top-20, yaw-set build, COLOR windows, publish.
With "pf" (a library built with -DMK_SCORE_TICKS=2): k_score_pf (the particle filter)'s
phases summed over its iterations: mask staging, particle poses, screened
tasks, unsure drain, per-particle sums, argmin.
With "color" (-DMK_SCORE_TICKS=3): COLOR's projection, row and sum phases.
usage: MANTIS_AMD_LIB=abvar/ticks.so python tools/score_ticks.py [pf | color] [rigs]"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main(rigs, pf=False, color=False):
    import mantis_amd as M
    from mantis_amd import synth

    W, H, CAMS, ND = 1280, 720, 4, 64
    K, D = synth.intrinsics(W, H)
    rng = np.random.default_rng(1000)
    ext = synth.rig_extrinsics(CAMS)
    cams, Tbc = [], []
    for r in range(ND):
        Twb = synth.random_base_pose(rng)
        for c in range(CAMS):
            Twc = Twb @ ext[c]
            cams.append(synth.make_cam(Twc[:3, :3], Twc[:3, 3], W, H))
            Tbc.append(ext[c])
    m = M.Mantis(max_cams=rigs * CAMS, max_width=W, max_height=H)
    m.set_map(*synth.load_map())
    fb = W * H * 3
    dev = m.device_alloc(len(cams) * fb)
    m.synth_render(cams, [synth.frame_seed(3, i) for i in range(len(cams))], dev)
    m.synchronize()
    n = rigs * CAMS
    imgs = [M.make_image(None, K, D, T_base_cam=Tbc[i % len(cams)], device_ptr=dev + (i % len(cams)) * fb,
                         width=W, height=H) for i in range(n)]
    m.process(imgs, rigs=rigs)
    m.process(imgs, rigs=rigs)
    tk = []
    for i in range(n):
        fc = m.frame_counters(i)
        if m.frame_debug(i).n_hyps > 0:
            tk.append(fc[10:16].astype(np.float64) * 0.01)  # 10 ns ticks -> us
    tk = np.array(tk)
    if color:  # MK_SCORE_TICKS=3: slots 1, 2 hold COLOR's projection / row phase ends
        for nm, a, b in (("COLOR project", 3, 1), ("COLOR rows", 1, 2), ("COLOR sums", 2, 4)):
            d = tk[:, b] - tk[:, a]
            print(f"{nm:14s} median {np.median(d):8.1f} us  p90 {np.percentile(d, 90):8.1f} us")
        m.close()
        return
    if pf:  # per-phase sums already
        d = tk
        tk = np.cumsum(tk, axis=1)
        names = ["staging", "particles", "tasks", "drain", "sums", "argmin"]
    else:
        d = np.diff(np.concatenate([np.zeros((len(tk), 1)), tk], 1), axis=1)
        names = ["shift tasks", "drain", "top-20", "yaw build", "COLOR", "publish"]
    for j, nm in enumerate(names):
        print(f"{nm:12s} median {np.median(d[:, j]):8.1f} us  p90 {np.percentile(d[:, j], 90):8.1f} us")
    print(f"total        median {np.median(tk[:, 5]):8.1f} us over {len(tk)} frames")
    m.close()


if __name__ == "__main__":
    a = sys.argv[1:]
    mode = a[0] if a and a[0] in ("pf", "color") else ""
    a = a[1:] if mode else a
    main(int(a[0]) if a else 256, mode == "pf", mode == "color")
