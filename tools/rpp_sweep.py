"""ObjPose queue study (GPU box): one context over the config-3 batch (1024
rigs x 4 cameras at 1280x720, the bench scene), stage times of rpp_first /
rpp_cand per setting BLOCKS[:ROUNDS[:SPILL]] (MANTIS_RPP_BLOCKS, and the tail
compaction's MANTIS_OP_ROUNDS / MANTIS_OP_SPILL; BLOCKS 0 = default grid),
plus the job and iteration counts of the two queues. One JSON line per setting.

    python tools/rpp_sweep.py 384:1 384:4:32 0:4:32 > gpurun_out/rpp_sweep.jsonl
"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main(settings):
    import mantis_amd as M
    from mantis_amd import synth

    W, H, CAMS, RIGS, ND = 1280, 720, 4, 1024, 128
    white, red, green = synth.load_map()
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
    nd = len(cams)
    fb = W * H * 3
    for s in settings:
        parts = s.split(":")
        env = dict(zip(("MANTIS_RPP_BLOCKS", "MANTIS_OP_ROUNDS", "MANTIS_OP_SPILL"), parts))
        if env.get("MANTIS_RPP_BLOCKS") == "0":
            del env["MANTIS_RPP_BLOCKS"]
        os.environ.update(env)
        m = M.Mantis(max_cams=RIGS * CAMS, max_width=W, max_height=H)
        m.set_map(white, red, green)
        dev = m.device_alloc(nd * fb)
        m.synth_render(cams, [synth.frame_seed(3, i) for i in range(nd)], dev)
        m.synchronize()
        imgs = [M.make_image(None, K, D, T_base_cam=Tbc[i % nd], device_ptr=dev + (i % nd) * fb, width=W, height=H)
                for i in range(RIGS * CAMS)]
        b = M.Batch(m, imgs, RIGS)
        b.run()
        m.set_profiling(True)
        acc = {}
        reps = 3
        t0 = time.perf_counter()
        for _ in range(reps):
            b.run()
            for k, v in m.stage_times():
                acc[k] = acc.get(k, 0.0) + v / reps
        el = (time.perf_counter() - t0) / reps
        m.set_profiling(False)
        it0 = it1 = nq = 0
        for i in range(RIGS * CAMS):
            fc = m.frame_counters(i)
            nq += int(fc[3])
            it0 += int(fc[16])
            it1 += int(fc[17])
        import hashlib
        dig = hashlib.sha1(b"".join(bytes(c) for c in b.cam_out)).hexdigest()[:16]
        line = {"setting": s, "step_ms": round(el * 1e3, 3), "first_jobs": nq, "iters": [it0, it1], "digest": dig,
                "stages_ms": {k: round(v, 3) for k, v in sorted(acc.items(), key=lambda kv: -kv[1])}}
        print(json.dumps(line), flush=True)
        m.close()
        for k in env:
            del os.environ[k]


if __name__ == "__main__":
    main(sys.argv[1:] or ["0:1", "0:4:32"])
