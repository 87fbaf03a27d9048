"""Single-rig latency with and without the hipGraph replay of the rig-latency
path (GPU box): one 4-camera 1280x720 rig of the bench scene per call,
device-resident frames, host submit -> result; median / p90 over the calls.
Run once per setting (MANTIS_GRAPHS=0 / default), each in its own process
(the switch is read at context creation, the packet-capture setting at HIP
start).

    python tools/p50_graph_ab.py [calls]
"""
import json
import os
import sys
import time

os.environ.setdefault("DEBUG_CLR_GRAPH_PACKET_CAPTURE", "0")

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main(calls):
    import mantis_amd as M
    from mantis_amd import synth

    W, H, CAMS, ND = 1280, 720, 4, 16
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
    m = M.Mantis(max_cams=CAMS, max_width=W, max_height=H, gn_enable=1)
    m.set_map(*synth.load_map())
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
    print(json.dumps({"graphs": os.environ.get("MANTIS_GRAPHS", "1") != "0" and
                      os.environ.get("DEBUG_CLR_GRAPH_PACKET_CAPTURE") == "0",
                      "calls": calls, "p50_ms": round(float(np.median(lat)), 3),
                      "p90_ms": round(float(np.percentile(lat, 90)), 3),
                      "min_ms": round(float(np.min(lat)), 3)}))
    m.close()


if __name__ == "__main__":
    main(int(sys.argv[1]) if len(sys.argv) > 1 else 64)
