"""Phase times of k_hyst_band (middle band of each frame; a library built with
-DMK_HYST_TICKS, MANTIS_AMD_LIB): one context, one batch of bench rigs;
median / p90 of each phase over the frames (wall clock: the block shares its
CU with others, so the phases' shares matter more than their sums).
Phases: planes to LDS, run counts + row bases, run extents + label init, row unions, finds + band flags, global writes + lists (the edge-word store after them is not timed).
With k_hyst_rec (the default path) the six values are instead: seam rounds,
most sweeps of one band, sweeps of all bands, row fills of all bands, first
settle and whole-kernel ticks.
usage: MANTIS_AMD_LIB=abvar/hticks.so python tools/hyst_ticks.py [rigs]"""
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
    if os.environ.get("MANTIS_HYST_REC", "1") != "0":
        v = np.array([m.frame_counters(i)[10:16] for i in range(n)], np.float64)
        names = ["seam rounds", "max sweeps/band", "sweeps (all)", "row fills", "settle us", "total us"]
        v[:, 4:] *= 0.01
        for j, nm in enumerate(names):
            print(f"{nm:16s} median {np.median(v[:, j]):9.1f}  p90 {np.percentile(v[:, j], 90):9.1f}  max {v[:, j].max():9.1f}")
        m.close()
        return
    tk = []
    for i in range(n):
        fc = m.frame_counters(i)
        tk.append(fc[10:16].astype(np.float64) * 0.01)  # 10 ns ticks -> us
    tk = np.array(tk)
    d = np.diff(np.concatenate([np.zeros((len(tk), 1)), tk], 1), axis=1)
    names = ["load", "counts+scan", "runs+init", "unions", "finds+flags", "writes+lists"]
    for j, nm in enumerate(names):
        print(f"{nm:12s} median {np.median(d[:, j]):8.1f} us  p90 {np.percentile(d[:, j], 90):8.1f} us")
    print(f"total        median {np.median(tk[:, 5]):8.1f} us over {len(tk)} frames")
    m.close()


if __name__ == "__main__":
    main(int(sys.argv[1]) if len(sys.argv) > 1 else 256)
