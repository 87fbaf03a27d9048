"""Fraction of the map's landmarks in frame for the scored hypotheses of bench
frames (FrameDebug.hyp_n over the landmark count): how much a per-iteration
cull of surely-out-of-frame landmarks could save the scorers.
usage: python tools/inframe_stats.py [rigs]"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main(rigs):
    import mantis_amd as M
    from mantis_amd import synth

    W, H, CAMS, ND = 1280, 720, 4, 64
    K, D = synth.intrinsics(W, H)
    white, red, green = synth.load_map()
    nl = len(white) + len(red) + len(green)
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
    m.set_map(white, red, green)
    fb = W * H * 3
    dev = m.device_alloc(len(cams) * fb)
    m.synth_render(cams, [synth.frame_seed(3, i) for i in range(len(cams))], dev)
    m.synchronize()
    imgs = [M.make_image(None, K, D, T_base_cam=Tbc[i % len(cams)], device_ptr=dev + (i % len(cams)) * fb, width=W,
                         height=H) for i in range(rigs * CAMS)]
    M.Batch(m, imgs, rigs).run()
    fr = []
    for i in range(rigs * CAMS):
        d = m.frame_debug(i)
        n = int(d.n_hyps)
        if n > 0:
            fr.append(np.array(d.hyp_n[:n], np.float64) / nl)
    a = np.concatenate(fr) if fr else np.zeros(1)
    print(f"landmarks {nl}; frames with hypotheses {len(fr)}; in-frame fraction per hypothesis: "
          f"mean {a.mean():.3f} median {np.median(a):.3f} p10 {np.percentile(a, 10):.3f} p90 {np.percentile(a, 90):.3f}")
    m.close()


if __name__ == "__main__":
    main(int(sys.argv[1]) if len(sys.argv) > 1 else 64)
