"""Border length statistics of the bench scene's frames (GPU box): per frame,
borders of at most 128 points (one lane each in k_frame_contours' DP) and
longer ones (one wave each), with their point totals; medians over frames.

    python tools/fc_stats.py [frames]
"""
import ctypes as C
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main(nf):
    import mantis_amd as M
    from mantis_amd import synth

    W, H = 1280, 720
    K, D = synth.intrinsics(W, H)
    rng = np.random.default_rng(1000)
    ext = synth.rig_extrinsics(4)
    cams = []
    for r in range((nf + 3) // 4):
        Twb = synth.random_base_pose(rng)
        for c in range(4):
            Twc = Twb @ ext[c]
            cams.append(synth.make_cam(Twc[:3, :3], Twc[:3, 3], W, H))
    cams = cams[:nf]
    m = M.Mantis(max_cams=nf, max_width=W, max_height=H)
    m.set_map(*synth.load_map())
    fb = W * H * 3
    dev = m.device_alloc(nf * fb)
    m.synth_render(cams, [synth.frame_seed(3, i) for i in range(nf)], dev)
    m.synchronize()
    ext4 = [ext[i % 4] for i in range(nf)]
    imgs = [M.make_image(None, K, D, T_base_cam=ext4[i], device_ptr=dev + i * fb, width=W, height=H) for i in range(nf)]
    m.process(imgs, rigs=nf // 4)
    rows = []
    for f in range(nf):
        c = np.array([len(p) for p, _ in m.contours(f)])
        s, l = c[c <= 128], c[c > 128]
        rows.append((len(c), len(s), int(s.sum()), len(l), int(l.sum()), int(l.max()) if len(l) else 0))
    a = np.array(rows)
    for j, nm in enumerate(["borders", "short (<=128)", "short points", "long (>128)", "long points", "longest"]):
        print(f"{nm:14s} median {np.median(a[:, j]):9.1f}  p90 {np.percentile(a[:, j], 90):9.1f}")
    m.close()


if __name__ == "__main__":
    main(int(sys.argv[1]) if len(sys.argv) > 1 else 64)
