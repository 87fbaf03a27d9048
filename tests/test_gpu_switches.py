"""Every run-time switch that selects a kernel path, fenced:
each setting's context processes the same rigs as a default context and must
return byte-identical rig results, camera results, frame records and cv::RNG
state. Two batch sizes, because the switches act on different paths: one
4-camera rig (<= CUs / 4 frames: the rig-latency kernels) and 20 rigs (80
frames: the throughput kernels). One setting per path is also held to the
oracle. Round 4's ObjPose job-duplication bug lived in exactly such a switch
path (ADVICE / VERDICT r05 weak item 6).

Switches tested elsewhere: MANTIS_OP_LANES_SMALL / _ROUNDS_SMALL
(test_small_batch_objpose_queue_settings), MANTIS_CANNY_STRIP, MANTIS_MORPH_WALK,
MANTIS_TRACE_LDS_FRAMES, MANTIS_SEG_M, MANTIS_SCREEN
(test_gpu_parity.py), MANTIS_PF_MASK_GLOBAL (test_gpu_pipeline.py),
MANTIS_HYST_REC, MANTIS_HYST_EPOCH0 (test_hysteresis.py).
"""
import os

import numpy as np
import pytest

import _oracle as O
from mantis_amd import synth
from test_gpu_parity import _cmp_debug

pytestmark = pytest.mark.gpu

W, H, CAMS = 1280, 720, 4


@pytest.fixture(scope="module")
def scene(landmark_map):
    """20 rigs x 4 cameras rendered once into HBM by a holder context (its
    allocation is valid for every context of the process on this device)."""
    import mantis_amd as M

    holder = M.Mantis(max_cams=1, max_width=W, max_height=H)
    K, D = synth.intrinsics(W, H)
    ext = synth.rig_extrinsics(CAMS)
    rng = np.random.default_rng(606)
    cams, tbc = [], []
    for r in range(20):
        Twb = synth.random_base_pose(rng)
        for c in range(CAMS):
            Twc = Twb @ ext[c]
            cams.append(synth.make_cam(Twc[:3, :3], Twc[:3, 3], W, H))
            tbc.append(ext[c])
    fb = W * H * 3
    dev = holder.device_alloc(len(cams) * fb)
    holder.synth_render(cams, [synth.frame_seed(6, i) for i in range(len(cams))], dev)
    holder.synchronize()
    imgs = [M.make_image(None, K, D, T_base_cam=tbc[i], device_ptr=dev + i * fb, width=W, height=H)
            for i in range(len(cams))]
    yield imgs, holder, dev, fb
    holder.close()


def _run(env, imgs, rigs, landmark_map):
    import mantis_amd as M

    saved = {k: os.environ.get(k) for k in env}
    os.environ.update(env)
    try:
        m = M.Mantis(max_cams=len(imgs), max_width=W, max_height=H)
    finally:
        for k, v in saved.items():
            if v is None:
                os.environ.pop(k)
            else:
                os.environ[k] = v
    try:
        m.set_map(*landmark_map)
        m.rng_state = 1
        rig, cams = m.process(imgs, rigs=rigs)
        n = len(imgs)
        return {"rig": [bytes(r) for r in rig], "cams": [bytes(c) for c in cams],
                "dbg": [bytes(m.frame_debug(f)) for f in range(n)], "rng": m.rng_state,
                "small": int(M.lib().mantis_small_batch_frames(m.h)),
                "records": [m.frame_debug(f) for f in range(min(n, 4))]}
    finally:
        m.close()


def _same(got, ref, tag):
    assert got["rng"] == ref["rng"], f"{tag}: cv::RNG state differs"
    assert got["rig"] == ref["rig"], f"{tag}: rig results differ"
    for f in range(len(ref["cams"])):
        assert got["cams"][f] == ref["cams"][f], f"{tag}: camera {f} result differs"
        assert got["dbg"][f] == ref["dbg"][f], f"{tag}: camera {f} frame record differs"


# (switch, value): the rig-latency path (one rig)
SMALL = [("MANTIS_PF_SPLIT", "0"),            # one particle-filter block per frame instead of the split kernels
         ("MANTIS_MORPH_WALK_SMALL", "16"),   # 16-row walker segments (45 per frame)
         ("MANTIS_MORPH_WALK_SMALL", "100000"),  # one segment per frame: the walker numbers the runs
         ("MANTIS_FC_SMALL_FRAMES", "0"),     # the throughput kernels on a one-rig batch
         ("MANTIS_RPP_BLOCKS", "1"),          # a one-block ObjPose grid (the small path sizes its own grid: no effect)
         ("MANTIS_GRAPHS", "0")]              # every kernel launched directly instead of the two replayed hipGraphs
# the throughput path (80 frames)
LARGE = [("MANTIS_RPP_BLOCKS", "8"),          # a small persistent ObjPose grid: every lane serves many jobs
         ("MANTIS_RPP_BLOCKS", "32"),
         ("MANTIS_OP_ROUNDS", "1"),           # no tail compaction
         ("MANTIS_OP_ROUNDS", "3"),
         ("MANTIS_OP_SPILL", "0"),            # a wave never hands its jobs on
         ("MANTIS_OP_SPILL", "64"),           # every wave with an idle lane hands its jobs on
         ("MANTIS_FC_SMALL_FRAMES", "100000"),  # the latency kernels on an 80-frame batch
         ("MANTIS_PF_SPLIT", "0"),            # (no effect on a large batch)
         ("MANTIS_CANNY_CAT", "0"),           # Canny strips per frame instead of over the frames side by side
         ("MANTIS_PF_SHIFTS", "0"),           # the 81 shifts in k_score_final instead of at the end of k_score_pf
         ("MANTIS_GN_FUSED", "0"),            # the rig GN as obs / acc / step kernels instead of one fused launch
         ("MANTIS_PF_INIT", "0"),             # k_score_init launched instead of its work at the start of k_score_pf
         ("MANTIS_PF_INIT", "2"),             # that work with its per-hypothesis arrays in global scratch
         ("MANTIS_SHIFT_SPLIT", "1"),         # the 81 shifts in k_score_shift_part blocks
         ("MANTIS_SHIFT_SPLIT", "0")]


def test_rig_latency_path_switches(scene, landmark_map):
    imgs = scene[0][:CAMS]
    ref = _run({}, imgs, 1, landmark_map)
    assert ref["small"] >= CAMS, "one rig must take the rig-latency kernels"
    for k, v in SMALL:
        _same(_run({k: v}, imgs, 1, landmark_map), ref, f"{k}={v} (one rig)")


def test_throughput_path_switches(scene, landmark_map):
    imgs = scene[0]
    ref = _run({}, imgs, len(imgs) // CAMS, landmark_map)
    assert ref["small"] < len(imgs), "80 frames must take the throughput kernels"
    for k, v in LARGE:
        _same(_run({k: v}, imgs, len(imgs) // CAMS, landmark_map), ref, f"{k}={v} (20 rigs)")


def test_switched_paths_against_oracle(scene, landmark_map):
    """The throughput kernels forced on one rig, and the latency kernels forced
    on the 20-rig batch (its first rig), against the CPU oracle frame by frame."""
    imgs, holder, dev, fb = scene
    K, D = synth.intrinsics(W, H)
    host = []
    for f in range(CAMS):
        b = np.empty((H, W, 3), np.uint8)
        holder.d2h(b, dev + f * fb)
        host.append(b)
    for env, batch in (({"MANTIS_FC_SMALL_FRAMES": "0"}, imgs[:CAMS]),
                       ({"MANTIS_FC_SMALL_FRAMES": "100000", "MANTIS_OP_ROUNDS": "1"}, imgs)):
        got = _run(env, batch, len(batch) // CAMS, landmark_map)
        orc = O.Oracle(*landmark_map, seed=1)
        for f in range(CAMS):
            _cmp_debug(got["records"][f], orc.process(host[f], K, D), f"{env} frame {f}")


def test_graph_replay_across_call_shapes(scene, landmark_map):
    """The rig-latency path replays captured hipGraphs (one pair per call shape):
    repeated calls, a call of another shape in between (a second capture) and
    the first shape again must give the same bytes as the first call, and the
    same as a context without graphs, including the cv::RNG state carried
    from call to call."""
    import mantis_amd as M

    imgs = scene[0]

    def calls(env):
        saved = {k: os.environ.get(k) for k in env}
        os.environ.update(env)
        try:
            m = M.Mantis(max_cams=8, max_width=W, max_height=H)
        finally:
            for k, v in saved.items():
                if v is None:
                    os.environ.pop(k)
                else:
                    os.environ[k] = v
        out = []
        try:
            m.set_map(*landmark_map)
            m.rng_state = 1
            for batch, rigs in ((imgs[:4], 1), (imgs[:4], 1), (imgs[4:12], 2), (imgs[8:12], 1), (imgs[:4], 1)):
                rig, cams = m.process(batch, rigs=rigs)
                out.append(([bytes(r) for r in rig], [bytes(c) for c in cams],
                            [bytes(m.frame_debug(f)) for f in range(len(batch))], m.rng_state))
        finally:
            m.close()
        return out

    g, d = calls({}), calls({"MANTIS_GRAPHS": "0"})
    assert len(g) == len(d)
    for k, (a, b) in enumerate(zip(g, d)):
        assert a == b, f"call {k}: graph replay differs from direct launches"
    # the same rig at another RNG state gives another particle filter, at the
    # same state the same bytes: the replays read the state-dependent inputs
    assert g[0][3] != g[1][3]


@pytest.mark.parametrize("wh", [(1280, 720), (992, 600), (1000, 600)])
def test_canny_strips_side_by_side(landmark_map, wh):
    """k_canny_strip<2> over the batch's frames laid side by side (W % 32 == 0:
    a strip may hold one frame's last columns and the next frame's first ones)
    against the per-frame strips and the oracle: 6 frames in one batch with
    the strip kernel forced on the small path (MANTIS_CANNY_STRIP=2). 992
    columns put the frame boundaries at a different place in every strip;
    1000 (W % 32 != 0) keeps the per-frame strips."""
    import mantis_amd as M

    Wc, Hc = wh
    K, D = synth.intrinsics(Wc, Hc)
    rng = np.random.default_rng(31)
    host = []
    for f in range(6):
        R, pos = synth.random_pose(rng)
        host.append(synth.render_host(synth.make_cam(R, pos, Wc, Hc), synth.frame_seed(7, f)))
    host[3] = np.clip(host[3].astype(np.int16) + rng.integers(-40, 40, host[3].shape), 0, 255).astype(np.uint8)
    imgs = [M.make_image(x, K, D) for x in host]

    def run(env):
        saved = {k: os.environ.get(k) for k in env}
        os.environ.update(env)
        try:
            m = M.Mantis(max_cams=6, max_width=Wc, max_height=Hc)
        finally:
            for k, v in saved.items():
                if v is None:
                    os.environ.pop(k)
                else:
                    os.environ[k] = v
        try:
            m.set_map(*landmark_map)
            m.rng_state = 1
            _, cams = m.process(imgs, rigs=6)
            return ([bytes(c) for c in cams], [bytes(m.frame_debug(f)) for f in range(6)],
                    [list(m.frame_counters(f)[:3]) for f in range(6)], [m.frame_debug(f) for f in range(6)])
        finally:
            m.close()

    per = run({"MANTIS_CANNY_STRIP": "2", "MANTIS_CANNY_CAT": "0"})
    cat = run({"MANTIS_CANNY_STRIP": "2"})
    assert cat[0] == per[0] and cat[1] == per[1] and cat[2] == per[2], f"{wh}: side-by-side strips differ"
    orc = O.Oracle(*landmark_map, seed=1)
    for f in range(6):
        _cmp_debug(cat[3][f], orc.process(host[f], K, D), f"{wh} frame {f}")
