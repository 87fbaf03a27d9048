"""Single-rig latency against the context's size and the contexts beside it
(GPU box): context 0 sized for `max_cams` frames, `extra` idle contexts of
4096 frames beside it (bench.py's default holds six), one 4-camera 1280x720
rig of the bench scene per call over 16 distinct rigs; median / p90.

    python tools/p50_ctx_probe.py max_cams extra [calls]
"""
import json
import os
import sys
import time

os.environ.setdefault("DEBUG_CLR_GRAPH_PACKET_CAPTURE", "0")

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main(max_cams, extra, calls):
    import mantis_amd as M
    from mantis_amd import synth

    W, H, CAMS = 1280, 720, 4
    ND = int(os.environ.get("P50_RIGS", "16"))
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
    maps = synth.load_map()
    m = M.Mantis(max_cams=max_cams, max_width=W, max_height=H, gn_enable=1, max_contour_points=98304)
    m.set_map(*maps)
    others = []
    for _ in range(extra):
        o = M.Mantis(max_cams=4096, max_width=W, max_height=H, gn_enable=1, max_contour_points=98304)
        o.set_map(*maps)
        others.append(o)
    fb = W * H * 3
    dev = m.device_alloc(len(cams) * fb)
    m.synth_render(cams, [synth.frame_seed(3, i) for i in range(len(cams))], dev)
    m.synchronize()
    imgs = [M.make_image(None, K, D, T_base_cam=Tbc[i], device_ptr=dev + i * fb, width=W, height=H)
            for i in range(len(cams))]
    for r in range(2):
        m.process(imgs[r * CAMS:(r + 1) * CAMS], rigs=1)
    lat = []
    for k in range(calls):
        one = imgs[(k % ND) * CAMS:(k % ND + 1) * CAMS]
        t0 = time.perf_counter()
        m.process(one, rigs=1)
        lat.append((time.perf_counter() - t0) * 1e3)
    print(json.dumps({"max_cams": max_cams, "extra_contexts": extra, "calls": calls,
                      "p50_ms": round(float(np.median(lat)), 3), "p90_ms": round(float(np.percentile(lat, 90)), 3),
                      "min_ms": round(float(np.min(lat)), 3)}), flush=True)
    for o in others:
        o.close()
    m.close()


if __name__ == "__main__":
    main(int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3]) if len(sys.argv) > 3 else 64)
