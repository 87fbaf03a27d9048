"""Phase ends of k_frame_contours per frame (FrameState.ticks, 10 ns, written
by the default build): one context, one batch of bench rigs; median / p90 of
each phase's duration. Phases: point-count scan, chunk compaction, short-
border approxPolyDP, long-border approxPolyDP, CCOMP order + duplicates,
quad filtering to the end.
usage: python tools/fc_ticks.py [rigs]"""
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
    tk = np.array([m.frame_counters(i)[10:16] for i in range(n)], np.float64) * 0.01
    d = np.diff(np.concatenate([np.zeros((n, 1)), tk], 1), axis=1)
    for j, nm in enumerate(["scan", "compaction", "approx short", "approx long", "ccomp + dups", "quads"]):
        print(f"{nm:14s} median {np.median(d[:, j]):8.1f} us  p90 {np.percentile(d[:, j], 90):8.1f}")
    print(f"{'total':14s} median {np.median(tk[:, 5]):8.1f} us")
    m.close()


if __name__ == "__main__":
    main(int(sys.argv[1]) if len(sys.argv) > 1 else 256)
