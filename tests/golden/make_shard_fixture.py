"""Writes tests/golden/shard_batch.npz: the per-frame records of a real
one-GPU batch for the CPU (gloo) tests of the camera-sharded bookkeeping
(tests/test_distributed.py). Run on the GPU box:

    python tests/golden/make_shard_fixture.py gpurun_out/shard_batch.npz

Batch: 3 rigs x 8 fisheye cameras at 1280x720 (the config-4 ring of
extrinsics at config-3 resolution), some cameras replaced by flat or noise
frames so not every frame reaches the particle filter (their flags are the
non-trivial input of the cross-rank cv::RNG offset rule), processed by
mantis_process_batch with rng_state 1, rig GN and weighting off (the rig result
is then exactly fuse + rng_state_after). Stored: every camera's
mantis_cam_result (raw bytes), T_base_cam, its reaches-PF flag, every rig's
mantis_result (raw bytes), and the cv::RNG states after k particle-filter frames
(k = 0..24, the oracle's cv::RNG restatement; 3000 gaussians per frame).
"""
import ctypes as C
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main(out):
    import _oracle as O
    import mantis_amd as M
    from mantis_amd import synth

    R_RIGS, CAMS, W, H = 3, 8, 1280, 720
    K, D = synth.intrinsics(W, H)
    ext = synth.rig_extrinsics(CAMS)
    rng = np.random.default_rng(8080)
    blank = {(0, 3): "flat", (1, 0): "noise", (1, 5): "flat", (2, 7): "noise"}
    imgs, tbc = [], []
    for r in range(R_RIGS):
        Twb = synth.random_base_pose(rng)
        for c in range(CAMS):
            kind = blank.get((r, c))
            if kind == "flat":
                img = np.full((H, W, 3), 90, np.uint8)
            elif kind == "noise":
                img = rng.integers(80, 120, (H, W, 3), dtype=np.uint8)
            else:
                Twc = Twb @ ext[c]
                img = synth.render_host(synth.make_cam(Twc[:3, :3], Twc[:3, 3], W, H), synth.frame_seed(9, r * CAMS + c))
            imgs.append(M.make_image(img, K, D, T_base_cam=ext[c]))
            tbc.append(ext[c])
    m = M.Mantis(max_cams=R_RIGS * CAMS, max_width=W, max_height=H, gn_enable=0, rig_weighting=0)
    m.set_map(*synth.load_map())
    m.rng_state = 1
    rigs, cams = m.process(imgs, rigs=R_RIGS)
    pf = np.array([int(m.frame_counters(i)[6]) for i in range(len(imgs))], np.int32)
    states = [1]
    s = 1
    for _ in range(len(imgs)):
        _, s = O.gaussians(s, 3000)
        states.append(s)
    assert rigs[-1].rng_state_after == states[int(pf.sum())]
    cam_bytes = np.stack([np.frombuffer(bytes(c), np.uint8) for c in cams])
    rig_bytes = np.stack([np.frombuffer(bytes(r), np.uint8) for r in rigs])
    np.savez_compressed(out, cam_bytes=cam_bytes, tbc=np.array(tbc), pf=pf, rig_bytes=rig_bytes,
                        states=np.array(states, np.uint64), per=np.int64(3000), rigs=np.int64(R_RIGS),
                        cams=np.int64(CAMS), cam_result_size=np.int64(C.sizeof(M.MantisCamResult)),
                        result_size=np.int64(C.sizeof(M.MantisResult)))
    print(f"shard fixture: {len(imgs)} frames, {int(pf.sum())} reach the particle filter, "
          f"published rigs {[r.publish for r in rigs]}")
    m.close()


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else os.path.join(ROOT, "tests", "golden", "shard_batch.npz"))
