"""GPU parity, second part: reference goldens through the C-ABI, the real
config-1 frame (test/grid1.jpg), config-4 resolution (1920x1080, contour
tracing without the LDS bitmap), multi-rig batches with rig fusion, and the
MFMA Gauss-Newton accumulator.

Tolerances: RPP poses 1e-9 absolute (device libm vs glibc ulps in atan2/acos/
sin/cos inside the 2nd-pose search; the decisions are exact); GN accumulators
1e-12 relative (MFMA f64 sums in a different order than numpy's matmul).
"""
import ctypes as C
import os

import numpy as np
import pytest

import _gn_ref as G
import _oracle as O
from mantis_amd import synth
from test_gpu_parity import POSE_TOL, _cmp_debug

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


@pytest.fixture(scope="module")
def m720(landmark_map):
    import mantis_amd as M

    m = M.Mantis(max_cams=8, max_width=1280, max_height=720)
    m.set_map(*landmark_map)
    yield m
    m.close()


def test_rpp_reference_golden_on_gpu(m720):
    d = np.load(os.path.join(GOLD, "rpp_golden.npz"), allow_pickle=False)
    ip = np.transpose(d["iprts"][:, :2, :], (0, 2, 1))
    op = np.transpose(d["model"], (0, 2, 1))
    R, t, e, st = m720.rpp(ip, op)
    assert np.array_equal(st, d["status"])
    np.testing.assert_allclose(R, d["R"], atol=POSE_TOL, rtol=0)
    np.testing.assert_allclose(t, d["t"], atol=POSE_TOL, rtol=0)
    np.testing.assert_allclose(e, d["errs"][:, :2], rtol=1e-9, atol=1e-15)


def test_grid1_config1_frame(m720, landmark_map):
    import mantis_amd as M

    g = np.load(os.path.join(GOLD, "grid1.npz"), allow_pickle=False)
    img = M.make_image(g["bgr"], g["K"], g["D"])
    quads = m720.detect_quads(img)
    assert np.array_equal(quads, g["quads"])
    orc = O.Oracle(*landmark_map, seed=1)
    m720.rng_state = 1
    rig, cams = m720.process([img], rigs=1)
    o = orc.process(g["bgr"], g["K"], g["D"])
    _cmp_debug(m720.frame_debug(0), o, "grid1")
    assert m720.rng_state == orc.rng_state == int(g["rng_state_after"])


def test_config4_1080p_frames(landmark_map):
    import mantis_amd as M

    W, H = 1920, 1080
    K, D = synth.intrinsics(W, H)
    m = M.Mantis(max_cams=2, max_width=W, max_height=H)
    m.set_map(*landmark_map)
    orc = O.Oracle(*landmark_map, seed=1)
    rng = np.random.default_rng(77)
    frames = []
    for f in range(2):
        R, pos = synth.random_pose(rng)
        frames.append(synth.render_host(synth.make_cam(R, pos, W, H), synth.frame_seed(4, f)))
    m.rng_state = 1
    m.process([M.make_image(fr, K, D) for fr in frames], rigs=2)
    for i, fr in enumerate(frames):
        _cmp_debug(m.frame_debug(i), orc.process(fr, K, D), f"1080p frame {i}")
    assert m.rng_state == orc.rng_state
    m.close()


def _quat_mat(q):
    x, y, z, w = q
    return np.array([[1 - 2 * (y * y + z * z), 2 * (x * y - z * w), 2 * (x * z + y * w)],
                     [2 * (x * y + z * w), 1 - 2 * (x * x + z * z), 2 * (y * z - x * w)],
                     [2 * (x * z - y * w), 2 * (y * z + x * w), 1 - 2 * (x * x + y * y)]])


def test_two_rig_batch_and_fusion(m720, landmark_map):
    import mantis_amd as M

    K, D = synth.intrinsics()
    ext = synth.rig_extrinsics(4)
    rng = np.random.default_rng(5)
    imgs, host = [], []
    for r in range(2):
        Twb = synth.random_base_pose(rng)
        for c in range(4):
            Twc = Twb @ ext[c]
            fr = synth.render_host(synth.make_cam(Twc[:3, :3], Twc[:3, 3]), synth.frame_seed(3, 10 * r + c))
            host.append(fr)
            imgs.append(M.make_image(fr, K, D, T_base_cam=ext[c]))
    m720.rng_state = 1
    orc = O.Oracle(*landmark_map, seed=1)
    rigs, cams = m720.process(imgs, rigs=2)
    states = []
    for i, fr in enumerate(host):
        _cmp_debug(m720.frame_debug(i), orc.process(fr, K, D), f"rig {i // 4} cam {i % 4}")
        states.append(orc.rng_state)
    assert rigs[0].rng_state_after == states[3] and rigs[1].rng_state_after == states[7]
    for r in range(2):
        cs = cams[4 * r: 4 * r + 4]
        pub = [i for i in range(4) if cs[i].publish]
        assert rigs[r].n_cams_published == len(pub)
        if not pub:
            continue
        b = min(pub, key=lambda i: (cs[i].error, i))
        Twc = np.eye(4)
        Twc[:3, :3] = _quat_mat(cs[b].orientation_xyzw)
        Twc[:3, 3] = cs[b].position
        Twb = Twc @ np.linalg.inv(ext[b])
        np.testing.assert_allclose(rigs[r].position, Twb[:3, 3], atol=1e-9)
        assert rigs[r].weight == cs[b].error and rigs[r].publish == 1


def test_gn_accumulate_mfma_vs_numpy(m720):
    import mantis_amd as M

    rng = np.random.default_rng(9)
    T = G.exp_se3_right(np.eye(4), np.array([0.1, 0.2, 1.3, 0.1, -0.2, 0.4]))
    ext = synth.rig_extrinsics(4)
    for n_per in (1, 5, 24, 61):
        obs = G.synth_rig_obs(rng, T, ext, n_per_cam=n_per, noise=1e-3)
        Tp = G.exp_se3_right(T, rng.normal(size=6) * 0.01)
        want = G.gn_accumulate(Tp, ext, obs)
        acc = np.zeros(28)
        Tc = np.ascontiguousarray(Tp)
        E = np.ascontiguousarray(np.array(ext))
        ob = np.ascontiguousarray(obs)
        st = M.lib().mantis_gn_accumulate(m720.h, Tc.ctypes.data, E.ctypes.data, len(ext), ob.ctypes.data, len(obs),
                                          acc.ctypes.data)
        assert st == 0
        np.testing.assert_allclose(acc, want, rtol=1e-12, atol=1e-14 * np.abs(want).max())


def test_dense_config5_argmin(m720, landmark_map):
    """Config 5 structure (shifts x yaws x perturbations) on the cleaned frame:
    device argmin == first minimum of the per-hypothesis errors, errors
    bit-identical to the oracle, and two shards + the exchange rule agree."""
    import mantis_amd as M
    from mantis_amd import dense

    rng = np.random.default_rng(31)
    R, pos = synth.random_pose(rng)
    K, D = synth.intrinsics()
    img = synth.render_host(synth.make_cam(R, pos), synth.frame_seed(5, 1))
    im = M.make_image(img, K, D)
    _, mask = m720.masks(im)
    hyps = dense.config5_hypotheses(R, pos, np.random.default_rng(3), n_particles=3)
    assert len(hyps) == 972
    err, npj = m720.score(im, hyps, fast=True, mask=mask)
    e, i = m720.score_argmin(im, hyps, 0, False, mask)
    assert i == int(np.argmin(err)) and e == err.min()
    cut = 500
    a = m720.score_argmin(im, hyps[:cut], 0, False, mask)
    b = m720.score_argmin(im, hyps[cut:], cut, False, mask)
    assert M.argmin_pick([a, b]) == (e, i)
    orc = O.Oracle(*landmark_map, seed=1)
    cleaned = img * (mask[..., None] != 0)
    oe, on = orc.score(cleaned, K, D, hyps[:200], fast=True)
    assert np.array_equal(err[:200], oe) and np.array_equal(npj[:200], on)


def test_rig_gn_refines_pose(landmark_map):
    """cfg.gn_enable (SURVEY a-21, config 3): the batched rig Gauss-Newton
    (one correspondence per quad: the crossing of its undistorted diagonals ->
    the grid cell centre it images; MFMA J^T J / J^T r, 6x6 Cholesky) equals
    its FP64 restatement (correspondences and pose to 1e-9), moves the fused
    base pose towards the synthetic ground truth and is reproducible run to
    run; with GN off the result is the reference fusion."""
    from test_gpu_multi import check_rig_gn_against_restatement
    import mantis_amd as M

    K, D = synth.intrinsics()
    ext = synth.rig_extrinsics(4)
    rng = np.random.default_rng(21)
    n_rigs = 6
    imgs, truth = [], []
    for r in range(n_rigs):
        Twb = synth.random_base_pose(rng)
        truth.append(Twb)
        for c in range(4):
            Twc = Twb @ ext[c]
            fr = synth.render_host(synth.make_cam(Twc[:3, :3], Twc[:3, 3]), synth.frame_seed(7, 10 * r + c))
            imgs.append(M.make_image(fr, K, D, T_base_cam=ext[c]))
    res = {}
    for gn in (0, 1):
        m = M.Mantis(M.default_config(max_cams=4 * n_rigs, max_width=1280, max_height=720, gn_enable=gn,
                                      gn_iterations=8))
        m.set_map(*landmark_map)
        s0 = m.rng_state
        res[gn] = m.process(imgs, rigs=n_rigs)[0]
        if gn:
            m.rng_state = s0  # same particle-filter stream, same fused poses
            again = m.process(imgs, rigs=n_rigs)[0]
            for a, b in zip(res[gn], again):
                assert list(a.position) == list(b.position) and list(a.orientation_xyzw) == list(b.orientation_xyzw)
            assert check_rig_gn_against_restatement(m, ext, n_rigs, K, D, 8) >= 3
        m.close()
    e0, e1 = [], []
    for r in range(n_rigs):
        p0 = np.array(res[0][r].position)
        p1 = np.array(res[1][r].position)
        pt = truth[r][:3, 3]
        if not res[0][r].publish or np.linalg.norm(p0 - pt) > 0.1:
            continue  # grid-periodic or yaw-ambiguous answer: GN refines around it, not towards the truth
        assert res[1][r].gn_iterations > 0 and np.isfinite(res[1][r].gn_cost)
        R1 = _quat_mat(res[1][r].orientation_xyzw)
        ang = np.degrees(np.arccos(np.clip((np.trace(R1.T @ truth[r][:3, :3]) - 1) / 2, -1, 1)))
        assert ang < 1.0
        e0.append(np.linalg.norm(p0 - pt))
        e1.append(np.linalg.norm(p1 - pt))
    assert len(e0) >= 3
    assert np.mean(e1) < np.mean(e0), (e0, e1)
    assert max(e1) < 0.02, e1


def test_ros_wire_callbacks_match_process(landmark_map):
    """The ROS side of the drop-in end to end (include/mantis_ros.h): the
    serialized sensor_msgs/Image + CameraInfo through mantis_ros_image_callback
    give the same frame result as mantis_process and the oracle's decision, and
    the serialized PoseWithCovarianceStamped carries it (frame "world", stamp 0
    as the reference); the mantisService request through
    mantis_ros_service_call answers with pose / weight / num_particles of the
    rig result."""
    import mantis_amd as M
    from mantis_amd import ros

    white, red, green = landmark_map
    K, D = synth.intrinsics()
    rng = np.random.default_rng(17)
    frames = []
    for f in range(3):
        R, pos = synth.random_pose(rng)
        frames.append(synth.render_host(synth.make_cam(R, pos), synth.frame_seed(4, f)))
    a = M.Mantis(max_cams=4)
    b = M.Mantis(max_cams=4)
    try:
        for m in (a, b):
            m.set_map(white, red, green)
            m.rng_state = 1
        orc = O.Oracle(white, red, green, seed=1)
        ci = ros.camera_info_bytes(np.asarray(K).reshape(9), list(D), 1280, 720)
        published = 0
        for img in frames:
            msg = ros.image_bytes(img, step=3 * 1280 + 32, stamp=(100, 200), frame_id="cam0")
            pose, cr = ros.image_callback(a, msg, ci)
            _, ref = b.process([M.make_image(img, K, D)])
            o = orc.process(img, K, D)
            assert cr.reason == ref[0].reason == o.reason and cr.publish == ref[0].publish == o.publish
            assert list(cr.position) == list(ref[0].position)
            assert np.allclose(list(cr.position), list(o.position), atol=1e-9)
            if cr.publish:
                published += 1
                d = ros.parse_pose_bytes(pose)
                assert d["frame_id"] == "world" and d["stamp"] == (0, 0)
                assert d["position"] == tuple(cr.position)
                assert d["orientation_xyzw"] == tuple(cr.orientation_xyzw)
                assert d["covariance"] == tuple(cr.covariance)
            else:
                assert pose is None
        assert a.rng_state == b.rng_state == orc.rng_state
        # mantisService: two cameras as one rig
        req = ros.service_request_bytes([ros.image_bytes(i) for i in frames[:2]], [ci, ci])
        resp, rr = ros.service_call(a, req)
        _, _ = b.process([M.make_image(i, K, D) for i in frames[:2]])
        d = ros.parse_service_response_bytes(resp)
        assert d["position"] == tuple(rr.position) and d["weight"] == rr.weight
        assert d["num_particles"] == rr.num_particles > 0
        assert a.rng_state == b.rng_state
    finally:
        a.close()
        b.close()


def test_quad_gn_stage_and_pipeline(m720, landmark_map):
    """Per-quad GN after RPP (SURVEY a-21: 4 corners <-> model square, N = 4
    per quad): the device stage entry (mantis_quad_gn, k_quad_gn) against the
    FP64 restatement (tests/_gn_ref.quad_gn_reference) and the host build of
    the same code, on synthetic problems and chained after mantis_rpp_batch;
    in the pipeline (cfg.quad_gn_iterations) the RPP poses of the hypotheses
    are refined and the frame still goes through to a published pose.
    Tolerance 1e-8: see test_host_logic.test_quad_gn_host_build_matches_restatement."""
    import _hostcheck as HC
    import mantis_amd as M

    rng = np.random.default_rng(21)
    img, obj, R0, t0, Rt, tt = G.quad_problems(rng, 256)
    R, t, steps, costs = m720.quad_gn(img, obj, R0, t0, 8)
    Rh, th, sh, c0h, c1h = HC.quad_gn(R0, t0, img, obj, 8)
    np.testing.assert_allclose(R, Rh, atol=1e-8, rtol=0)
    np.testing.assert_allclose(t, th, atol=1e-8, rtol=0)
    np.testing.assert_allclose(costs[:, 0], c0h, rtol=1e-12)
    assert np.all(costs[:, 1] <= costs[:, 0])
    for i in range(0, 256, 8):
        Rr, tr, _, c0r, _ = G.quad_gn_reference(R0[i], t0[i], img[i], obj[i], 8)
        np.testing.assert_allclose(R[i], Rr, atol=1e-8, rtol=0)
        np.testing.assert_allclose(t[i], tr, atol=1e-8, rtol=0)
    # RPP -> GN chain on the same corners
    Rp, tp, e, st = m720.rpp(img, obj)
    ok = st >= 0
    R2, t2, s2, c2 = m720.quad_gn(img[ok], obj[ok], Rp[ok], tp[ok], 8)
    assert np.all(c2[:, 1] <= c2[:, 0] * (1 + 1e-12))
    for i in np.flatnonzero(ok)[:16]:
        j = int(np.sum(ok[:i]))
        Rr, tr, _, _, _ = G.quad_gn_reference(Rp[i], tp[i], img[i], obj[i], 8)
        np.testing.assert_allclose(t2[j], tr, atol=1e-8, rtol=0)
    # in the pipeline
    K, D = synth.intrinsics()
    R_wc, pos = synth.random_pose(np.random.default_rng(5))
    fr = synth.render_host(synth.make_cam(R_wc, pos), synth.frame_seed(2, 77))
    im = M.make_image(fr, K, D)
    out = {}
    for its in (0, 6):
        m = M.Mantis(M.default_config(max_cams=1, quad_gn_iterations=its))
        m.set_map(*landmark_map)
        m.rng_state = 1
        rig, cams = m.process([im])
        d = m.frame_debug(0)
        out[its] = (cams[0], d.n_hyps, np.array(d.hyp_c2w)[: d.n_hyps].copy())
        m.close()
    (c0_, n0, h0), (c6, n6, h6) = out[0], out[6]
    assert n0 > 0 and n6 > 0
    assert c6.status == 0 and c6.reason in (0, 3)
    # refined hypotheses stay next to the RPP ones (same quads, same clusters)
    if n0 == n6:
        assert np.max(np.abs(h6[:, 9:] - h0[:, 9:])) < 0.05
        assert np.any(h6 != h0)


def _quat_mat_xyzw(q):
    x, y, z, w = q
    return np.array([[1 - 2 * (y * y + z * z), 2 * (x * y - z * w), 2 * (x * z + y * w)],
                     [2 * (x * y + z * w), 1 - 2 * (x * x + z * z), 2 * (y * z - x * w)],
                     [2 * (x * z - y * w), 2 * (y * z + x * w), 1 - 2 * (x * x + y * y)]])


def test_rig_weighting_legacy_montecarlo(landmark_map):
    """cfg.rig_weighting = 1 (SURVEY f-4): every published camera's base pose
    is weighted over all 4 cameras of the rig with the legacy
    MonteCarlo::computeCameraError (MonteCarlo.cpp:183-226): the per-camera
    (error sum, count) of every (candidate, camera) job equals the oracle's
    restatement bit for bit, the weights are the per-camera errors' mean, the
    lowest weight wins and its base pose is the rig answer; a one-rank
    camera-sharded call (RCCL all-reduce of the slots) gives the same."""
    import mantis_amd as M

    K, D = synth.intrinsics()
    ext = synth.rig_extrinsics(4)
    rng = np.random.default_rng(33)
    n_rigs = 4
    imgs, frames = [], []
    for r in range(n_rigs):
        Twb = synth.random_base_pose(rng)
        for c in range(4):
            Twc = Twb @ ext[c]
            fr = synth.render_host(synth.make_cam(Twc[:3, :3], Twc[:3, 3]), synth.frame_seed(8, 10 * r + c))
            frames.append(fr)
            imgs.append(M.make_image(fr, K, D, T_base_cam=ext[c]))
    cfg = dict(max_cams=4 * n_rigs, max_width=1280, max_height=720)
    m0 = M.Mantis(M.default_config(**cfg))
    m0.set_map(*landmark_map)
    base, cams0 = m0.process(imgs, rigs=n_rigs)
    m0.close()
    m = M.Mantis(M.default_config(rig_weighting=1, **cfg))
    m.set_map(*landmark_map)
    rig, cams = m.process(imgs, rigs=n_rigs)
    for a, b in zip(cams0, cams):
        assert bytes(a) == bytes(b)  # the per-camera path is untouched
    orc = O.Oracle(*landmark_map, seed=1)
    checked = 0
    for r in range(n_rigs):
        w, c2w, sums, chosen = m.rig_weights(r, 4)
        cr = cams[4 * r: 4 * r + 4]
        pub = [k for k in range(4) if cr[k].publish]
        assert [k for k in range(5) if w[k] < np.finfo(np.float64).max] == pub  # slot 4: no motion prediction
        if not pub:
            assert chosen == -1
            assert bytes(rig[r]) == bytes(base[r])
            continue
        for k in pub:
            Twc = np.eye(4)
            Twc[:3, :3] = _quat_mat_xyzw(cr[k].orientation_xyzw)
            Twc[:3, 3] = cr[k].position
            Twb = Twc @ np.linalg.inv(ext[k])
            tot = 0.0
            for c in range(4):
                Tcw = np.linalg.inv(Twb @ ext[c])
                np.testing.assert_allclose(c2w[k, c], np.concatenate([Tcw[:3, :3].reshape(9), Tcw[:3, 3]]),
                                           atol=1e-12, rtol=0)
                o = orc.camera_error(frames[4 * r + c], K, D, c2w[k, c])
                assert np.array_equal(o[0], sums[k, c]), (r, k, c, o, sums[k, c])
                e, n = sums[k, c]
                tot += (1e17 if n < 10 else e) / n
            assert tot / 4 == w[k]
        assert chosen == min(pub, key=lambda k: (w[k], k))
        assert rig[r].weight == w[chosen] and rig[r].publish == 1
        Twc = np.eye(4)
        Twc[:3, :3] = _quat_mat_xyzw(cr[chosen].orientation_xyzw)
        Twc[:3, 3] = cr[chosen].position
        np.testing.assert_allclose(rig[r].position, (Twc @ np.linalg.inv(ext[chosen]))[:3, 3], atol=1e-9)
        checked += 1
    assert checked >= 2
    ms = M.Mantis(M.default_config(rig_weighting=1, **cfg))
    ms.set_map(*landmark_map)
    ms.comm_init(0, 1)
    rs, _ = ms.process_sharded(imgs, n_rigs, [0, 1, 2, 3], 4)
    for a, b in zip(rig, rs):
        assert bytes(a) == bytes(b)
    for r in range(n_rigs):
        a, b = m.rig_weights(r, 4), ms.rig_weights(r, 4)
        assert np.array_equal(a[0], b[0]) and np.array_equal(a[2], b[2]) and a[3] == b[3]
    m.close()
    ms.close()


def test_service_motion_prediction(landmark_map):
    """mantisService motion (srv/mantisService.srv:4-8, include/mantis.h
    mantis_process): the context keeps the last published rig pose; with a
    delta the prediction T_prior * Delta joins the rig candidates and is
    re-evaluated with the legacy weighting -- its world->camera poses are the
    composition, its per-camera sums equal the oracle's computeCameraError, and
    the winner is the lowest weight. An unset motion (zero quaternion), or no
    prior, leaves the reference callback's answer unchanged."""
    import mantis_amd as M

    K, D = synth.intrinsics()
    ext = synth.rig_extrinsics(4)
    rng = np.random.default_rng(44)
    T0 = synth.random_base_pose(rng)
    delta = np.eye(4)
    delta[:3, :3] = synth.rot_z(0.03)
    delta[:3, 3] = [0.05, -0.02, 0.0]
    T1 = T0 @ delta
    rigs = []
    for r, T in enumerate((T0, T1)):
        fr = [synth.render_host(synth.make_cam((T @ ext[c])[:3, :3], (T @ ext[c])[:3, 3]), synth.frame_seed(9, 10 * r + c))
              for c in range(4)]
        rigs.append((fr, [M.make_image(f, K, D, T_base_cam=ext[c]) for c, f in enumerate(fr)]))
    m = M.Mantis(max_cams=4)
    m.set_map(*landmark_map)
    assert m.prior_pose is None
    r0, _ = m.process_motion(rigs[0][1], [0.1, 0, 0], [0, 0, 0, 1])  # no prior yet: plain callback
    if not r0.publish:
        pytest.skip("first rig not published")
    P = m.prior_pose
    np.testing.assert_allclose(P[:3, 3], r0.position, atol=0)
    # an unset motion is no motion
    s = m.rng_state
    a, ca = m.process_motion(rigs[1][1], [0, 0, 0], [0, 0, 0, 0])
    m.prior_pose = P
    m.rng_state = s
    b, cb = m.process_motion(rigs[1][1])
    assert bytes(a) == bytes(b)
    # with the delta: the prediction is weighted with the cameras' candidates
    m.prior_pose = P
    m.rng_state = s
    q = [0, 0, np.sin(0.015), np.cos(0.015)]
    res, cams = m.process_motion(rigs[1][1], delta[:3, 3], q)
    w, c2w, sums, chosen = m.rig_weights(0, 4)
    assert w[4] < np.finfo(np.float64).max
    Dm = np.eye(4)
    Dm[:3, :3] = _quat_mat_xyzw(q)
    Dm[:3, 3] = delta[:3, 3]
    pred = P @ Dm
    orc = O.Oracle(*landmark_map, seed=1)
    tot = 0.0
    for c in range(4):
        Tcw = np.linalg.inv(pred @ ext[c])
        np.testing.assert_allclose(c2w[4, c], np.concatenate([Tcw[:3, :3].reshape(9), Tcw[:3, 3]]), atol=1e-12)
        o = orc.camera_error(rigs[1][0][c], K, D, c2w[4, c])
        assert np.array_equal(o[0], sums[4, c])
        e, n = sums[4, c]
        tot += (1e17 if n < 10 else e) / n
    assert tot / 4 == w[4]
    valid = [k for k in range(5) if w[k] < np.finfo(np.float64).max]
    assert chosen == min(valid, key=lambda k: (w[k], k))
    assert res.weight == w[chosen]
    if chosen == 4:
        np.testing.assert_allclose(res.position, pred[:3, 3], atol=1e-12)
    # the prediction is near the truth of the second rig
    assert np.linalg.norm(pred[:3, 3] - T1[:3, 3]) < 0.1
    m.prior_pose = None
    m.rng_state = s
    c_, _ = m.process_motion(rigs[1][1], delta[:3, 3], q)
    assert bytes(c_) == bytes(b)
    m.close()


def test_dense_config5_full_grid_8_shards(m720, landmark_map):
    """Config 5 at its full size: 81 shifts x 4 yaws x 50 perturbations =
    16,200 hypotheses x 720 landmarks. The device argmin equals the first
    minimum of the per-hypothesis errors; the 8-shard split of BASELINE
    config 5 (2,025 per rank) combined by the cross-rank rule (what the RCCL
    all-gather feeds every rank) gives the same winner; a sample of 400
    hypotheses (every 40th, plus the winner) is bit-identical to the oracle."""
    import mantis_amd as M
    from mantis_amd import dense

    rng = np.random.default_rng(77)
    R, pos = synth.random_pose(rng)
    K, D = synth.intrinsics()
    img = synth.render_host(synth.make_cam(R, pos), synth.frame_seed(5, 2))
    im = M.make_image(img, K, D)
    _, mask = m720.masks(im)
    hyps = dense.config5_hypotheses(R, pos, np.random.default_rng(5))
    assert len(hyps) == 16200
    err, npj = m720.score(im, hyps, fast=True, mask=mask)
    e, i = m720.score_argmin(im, hyps, 0, False, mask)
    assert i == int(np.argmin(err)) and e == err.min()
    # device-resident inputs (mantis_score_argmin_dev): the same winner
    d_h = m720.device_alloc(hyps.nbytes)
    d_m = m720.device_alloc(mask.nbytes)
    try:
        m720.h2d(d_h, np.ascontiguousarray(hyps, np.float64))
        m720.h2d(d_m, np.ascontiguousarray(mask, np.uint8))
        assert m720.score_argmin_dev(im, d_h, len(hyps), 0, False, d_m) == (e, i)
    finally:
        m720.device_free(d_h)
        m720.device_free(d_m)
    pairs = []
    for r in range(8):
        lo, hi = dense.shard_range(len(hyps), r, 8)
        assert hi - lo == 2025
        pairs.append(m720.score_argmin(im, hyps[lo:hi], lo, False, mask))
    assert M.argmin_pick(pairs) == (e, i)
    orc = O.Oracle(*landmark_map, seed=1)
    cleaned = img * (mask[..., None] != 0)
    sel = np.unique(np.concatenate([np.arange(0, 16200, 40), [i]]))
    oe, on = orc.score(cleaned, K, D, hyps[sel], fast=True)
    assert np.array_equal(err[sel], oe) and np.array_equal(npj[sel], on)


def test_pf_mask_lds_and_global_paths_agree(landmark_map):
    """k_score_pf reads the clean mask from an LDS copy of the frame's tiled
    plane when it fits (720p) and through the L1 otherwise
    (MANTIS_PF_MASK_GLOBAL=1 forces that path); both block shapes (the
    small-batch 1024-thread one and the large-batch 640-thread one, chosen by
    MANTIS_TRACE_LDS_FRAMES) must give bit-identical frame results."""
    import os

    import mantis_amd as M

    K, D = synth.intrinsics()
    rng = np.random.default_rng(23)
    frames = []
    for f in range(4):
        R, pos = synth.random_pose(rng)
        frames.append(M.make_image(synth.render_host(synth.make_cam(R, pos), synth.frame_seed(6, f)), K, D))

    def run(env):
        old = {k: os.environ.get(k) for k in env}
        os.environ.update(env)
        try:
            m = M.Mantis(max_cams=4)
        finally:
            for k, v in old.items():
                if v is None:
                    os.environ.pop(k, None)
                else:
                    os.environ[k] = v
        try:
            m.set_map(*landmark_map)
            m.rng_state = 1
            _, cams = m.process(frames)
            return [(c.reason, c.publish, c.pf_error, tuple(c.position), tuple(c.orientation_xyzw)) for c in cams]
        finally:
            m.close()

    for small in ("64", "0"):
        lds = run({"MANTIS_TRACE_LDS_FRAMES": small})
        glob = run({"MANTIS_TRACE_LDS_FRAMES": small, "MANTIS_PF_MASK_GLOBAL": "1"})
        assert lds == glob, small
        assert any(r[0] >= 0 for r in lds)


def test_dense_batch_matches_per_frame(m720, landmark_map):
    """mantis_score_argmin_batch (config 5 batched: one launch over several
    frames' hypothesis blocks, per-frame argmins, device-resident inputs)
    equals mantis_score_argmin per frame -- uneven block sizes, an empty
    block, a frame without a mask -- also through the one-rank RCCL exchange."""
    import mantis_amd as M
    from mantis_amd import dense

    K, D = synth.intrinsics()
    rng = np.random.default_rng(97)
    imgs, hyps, masks = [], [], []
    for f in range(4):
        R, pos = synth.random_pose(rng)
        img = synth.render_host(synth.make_cam(R, pos), synth.frame_seed(5, 10 + f))
        im = M.make_image(img, K, D)
        imgs.append(im)
        masks.append(m720.masks(im)[1])
        hyps.append(dense.config5_hypotheses(R, pos, np.random.default_rng(f), n_particles=2 + f))
    hyps[2] = hyps[2][:0]  # an empty block
    bases = [0, 5000, 10, 77]
    want = []
    for f in range(4):
        if len(hyps[f]) == 0:
            want.append((np.finfo(np.float64).max, -1))
            continue
        want.append(m720.score_argmin(imgs[f], hyps[f], bases[f], False, masks[f] if f != 3 else None))
    ptrs = []
    try:
        d_h = [m720.device_alloc(max(8, h.nbytes)) for h in hyps]
        d_m = [m720.device_alloc(mk.nbytes) for mk in masks]
        ptrs = d_h + d_m
        for f in range(4):
            if len(hyps[f]):
                m720.h2d(d_h[f], np.ascontiguousarray(hyps[f], np.float64))
            m720.h2d(d_m[f], np.ascontiguousarray(masks[f], np.uint8))
        mptr = [d_m[0], d_m[1], d_m[2], 0]
        got = m720.score_argmin_batch(imgs, d_h, [len(h) for h in hyps], bases, False, mptr)
        for f in range(4):
            if want[f][1] < 0:
                assert got[f][1] == -1
            else:
                assert got[f] == want[f], f"frame {f}: {got[f]} vs {want[f]}"
        mc = M.Mantis(max_cams=8, max_width=1280, max_height=720)
        try:
            mc.set_map(*landmark_map)
            mc.comm_init(0, 1)
            dh2 = [mc.device_alloc(max(8, h.nbytes)) for h in hyps]
            dm2 = [mc.device_alloc(mk.nbytes) for mk in masks]
            for f in range(4):
                if len(hyps[f]):
                    mc.h2d(dh2[f], np.ascontiguousarray(hyps[f], np.float64))
                mc.h2d(dm2[f], np.ascontiguousarray(masks[f], np.uint8))
            got2 = mc.score_argmin_batch(imgs, dh2, [len(h) for h in hyps], bases, True, [dm2[0], dm2[1], dm2[2], 0])
            assert got2 == got
            # rank-local failures go through the agreement all-reduce before the
            # all-gather (with more ranks the others return MANTIS_ERR_COMM
            # instead of blocking in it); the communicator stays usable
            bad = list(imgs)
            bad[1] = M.make_image(np.zeros((720, 1280, 3), np.uint8), K, D)
            bad[1].step_bytes = 3 * 1280 - 3
            with pytest.raises(M.MantisError, match="step"):
                mc.score_argmin_batch(bad, dh2, [len(h) for h in hyps], bases, True, [dm2[0], dm2[1], dm2[2], 0])
            with pytest.raises(M.MantisError, match="hypothesis block"):
                mc.score_argmin_batch(imgs, dh2, [len(h) for h in hyps[:3]] + [-1], bases, True,
                                      [dm2[0], dm2[1], dm2[2], 0])
            with pytest.raises(M.MantisError, match="step"):
                mc.score_argmin(bad[1], hyps[0], 0, True, masks[0])
            assert mc.score_argmin_batch(imgs, dh2, [len(h) for h in hyps], bases, True,
                                         [dm2[0], dm2[1], dm2[2], 0]) == got
            assert mc.score_argmin(imgs[0], hyps[0], bases[0], True, masks[0]) == want[0]
        finally:
            mc.close()
    finally:
        for p in ptrs:
            m720.device_free(p)


def test_rpp_fault_golden_on_gpu(m720):
    """Fault injection, RPP: the degenerate problems of
    tests/golden/rpp_faults.npz (regression outputs of the oracle's RPP restatement) through
    the device RPP (mantis_rpp_batch): status 0 where Rpp() returns false (no
    2nd-pose candidate: the first ObjPose's pose is kept, RPP.cpp:13-64) and the
    reference's R, t and errors."""
    d = np.load(os.path.join(GOLD, "rpp_faults.npz"), allow_pickle=False)
    ip = np.transpose(d["iprts"][:, :2, :], (0, 2, 1))
    op = np.transpose(d["model"], (0, 2, 1))
    R, t, e, st = m720.rpp(ip, op)
    assert (d["status"] == 0).sum() >= 40
    assert np.array_equal(st, d["status"])
    stable = _rpp_stable(d)
    assert stable.sum() >= 12  # the centred squares and huge spreads
    np.testing.assert_allclose(R[stable], d["R"][stable], atol=POSE_TOL, rtol=0)
    np.testing.assert_allclose(t[stable], d["t"][stable], atol=POSE_TOL, rtol=0)
    np.testing.assert_allclose(e[stable], d["errs"][stable, :2], rtol=1e-9, atol=1e-15)
    # rank-deficient problems (collinear, repeated, coincident points, 1e-7
    # spreads): the reference's own pose moves by O(1) when an input moves by
    # one ulp (_rpp_stable), so a 1-ulp difference of a device libm call picks
    # another, equally valid, minimiser. There: a rotation, and errors that are
    # the reference's error formulas (RPP.cpp ObjPose: object-space error over
    # the line-of-sight projectors; image error against the FIRST image point,
    # the reference's Qp(0,0) indexing) evaluated at the returned pose.
    for k in np.flatnonzero(~stable):
        Rk = R[k]
        np.testing.assert_allclose(Rk.T @ Rk, np.eye(3), atol=1e-9, err_msg=str(d["name"][k]))
        m = d["model"][k]
        v = d["iprts"][k]
        q = Rk @ m + t[k][:, None]
        oe = 0.0
        for i in range(m.shape[1]):
            F = np.outer(v[:, i], v[:, i]) / (v[:, i] @ v[:, i])
            oe += np.sum(((np.eye(3) - F) @ q[:, i]) ** 2)
        ie = np.sum((q[0] / q[2] - v[0, 0]) ** 2 + (q[1] / q[2] - v[1, 0]) ** 2)
        n = m.shape[1]
        np.testing.assert_allclose(e[k], [np.sqrt(oe / n), np.sqrt(ie / n)], rtol=1e-6, atol=1e-9,
                                   err_msg=str(d["name"][k]))


def _rpp_stable(d, trials=12):
    """Problems whose reference pose is stable to rounding: the oracle (bit-
    exact with the reference on these problems, test_oracle_pins) moves by less
    than 1e-9 under 1-ulp relative perturbations of the image points."""
    rng = np.random.default_rng(1)
    out = np.ones(len(d["model"]), bool)
    for k in range(len(d["model"])):
        for _ in range(trials):
            ip = d["iprts"][k].copy()
            ip[:2] *= 1 + rng.normal(size=ip[:2].shape) * 2e-16
            _, Rk, tk, _, _ = O.rpp(d["model"][k], ip)
            if max(np.abs(Rk.reshape(3, 3) - d["R"][k]).max(), np.abs(tk - d["t"][k]).max()) > 1e-9:
                out[k] = False
                break
    return out


def _irregular_quads_frame(rng, W=640, H=480):
    """Dark, strongly non-square quadrilaterals on a light floor: the detector
    finds 4-vertex contours, but RPP's square model fits them so badly that
    every hypothesis fails the img_err > MAX_QUAD_ERROR gate
    (HypothesisGeneration.h:80-85) -> no hypotheses (src/mantis3.cpp:94-97)."""
    import PIL.Image
    import PIL.ImageDraw

    im = PIL.Image.fromarray(np.full((H, W, 3), 200, np.uint8))
    dr = PIL.ImageDraw.Draw(im)
    for _ in range(6):
        cx, cy = rng.uniform(80, W - 80), rng.uniform(80, H - 80)
        pts = [(cx + rng.uniform(-70, 70) * 2.5, cy + rng.uniform(-70, 70) * 0.3) for _ in range(4)]
        pts = sorted(pts, key=lambda p: np.arctan2(p[1] - cy, p[0] - cx))
        dr.polygon(pts, fill=(30, 30, 30))
    return np.asarray(im).copy()


def test_reason2_frames_match_oracle(landmark_map):
    """Fault injection, pipeline: frames whose quads all fail the hypothesis
    gate return reason 2 (no hypotheses, src/mantis3.cpp:94-97), publish
    nothing and draw no gaussians -- in a batch with normal frames, whose
    particle filters then read the cv::RNG stream where the sequential
    reference does."""
    import mantis_amd as M

    rng = np.random.default_rng(5)
    K, D = synth.intrinsics(640, 480)
    seq, reasons = [], []
    while len(seq) < 3:
        img = _irregular_quads_frame(rng)
        o = O.Oracle(*landmark_map, seed=1).process(img, K, D)
        if o.reason == 2 and o.n_quads > 0:
            seq.append(img)
    R, pos = synth.random_pose(np.random.default_rng(8))
    normal = synth.render_host(synth.make_cam(R, pos, 640, 480), synth.frame_seed(13, 0))
    seq = [seq[0], normal, seq[1], seq[2], normal]
    m = M.Mantis(max_cams=5, max_width=640, max_height=480)
    try:
        m.set_map(*landmark_map)
        m.rng_state = 1
        _, cams = m.process([M.make_image(img, K, D) for img in seq], rigs=5)
        orc = O.Oracle(*landmark_map, seed=1)
        for i, img in enumerate(seq):
            o = orc.process(img, K, D)
            _cmp_debug(m.frame_debug(i), o, f"frame {i}")
            assert cams[i].reason == o.reason and cams[i].publish == o.publish
            reasons.append(o.reason)
        assert reasons.count(2) == 3 and reasons[1] not in (1, 2)
        assert m.rng_state == orc.rng_state
    finally:
        m.close()


def test_reason4_no_green_landmarks_match_oracle(landmark_map):
    """Fault injection, yaw stage: with a map whose green set is empty every
    COLOR yaw set averages DBL_MAX, so determineBestYaw picks nothing -- the
    reference then reads hyps.back() of an empty set (UB); here
    reason 4 (no yaw), no publish -- identical to the oracle, and the fast
    scoring / particle filter before it is unchanged."""
    import mantis_amd as M

    white, red, green = landmark_map
    no_green = green[:0]
    K, D = synth.intrinsics()
    rng = np.random.default_rng(14)
    seq = []
    for f in range(3):
        R, pos = synth.random_pose(rng)
        seq.append(synth.render_host(synth.make_cam(R, pos), synth.frame_seed(14, f)))
    m = M.Mantis(max_cams=3, max_width=1280, max_height=720)
    try:
        m.set_map(white, red, no_green)
        m.rng_state = 1
        _, cams = m.process([M.make_image(img, K, D) for img in seq], rigs=3)
        orc = O.Oracle(white, red, no_green, seed=1)
        n4 = 0
        for i, img in enumerate(seq):
            o = orc.process(img, K, D)
            assert cams[i].reason == o.reason and cams[i].publish == o.publish == 0
            n4 += o.reason == 4
            g = m.frame_debug(i)
            assert g.n_hyps == o.n_hyps and g.pf_err == o.pf_err
            np.testing.assert_array_equal(np.array(g.shift_err), np.array(o.shift_err))
            assert g.yaw_best == o.yaw_best == -1
        assert n4 == 3
        assert m.rng_state == orc.rng_state
    finally:
        m.close()


def _debug_valid(d):
    """The parts of a frame debug record a call writes: the counts, the
    count-delimited quads / hypotheses, and the scoring fields only for frames
    that reach scoring (the rest of the record keeps earlier calls' bytes)."""
    n, c = d.n_quads, d.n_hyps
    out = [(d.reason, d.publish, d.n_raw_quads, n, d.n_gen, c),
           np.array(d.quads)[:n].tobytes(), np.array(d.test_pts)[:n].tobytes()]
    if d.reason not in (1, 2):
        out += [np.array(d.hyp_c2w)[:c].tobytes(), np.array(d.hyp_err)[:c].tobytes(), np.array(d.hyp_n)[:c].tobytes()]
        for f in ("best1_c2w", "pf_c2w", "pf_iter_err", "shift_err", "top20_err", "yaw_err", "pub_c2w", "position",
                  "orientation_xyzw", "covariance"):
            out.append(np.array(getattr(d, f)).tobytes())
        out.append((d.best1_err, d.pf_err, d.yaw_best, d.min_yaw_diff, d.pub_error, d.rng_state_after, d.n_scored))
    return out


@pytest.mark.parametrize("iters", [10, 0])
def test_throughput_and_latency_kernel_paths_agree(landmark_map, iters):
    """Batches above CUs / 4 frames take the throughput kernels (strip Canny,
    the morphology walker that numbers the runs, the L2 border walks, 256-thread
    contour blocks, one particle-filter block per frame); one rig at a time
    takes the latency ones (tile Canny, segmented walker + run kernels, LDS
    border walks, 1024-thread contour blocks, the filter's iterations split over
    blocks), which the oracle tests cover. The same 72 rendered frames through
    both: every camera result, frame record and the cv::RNG state bit-identical.
    iterations = 0 (no filter iteration: the one-block kernel's end-of-filter
    writes on both paths) as well as the default 10."""
    import mantis_amd as M

    W, H, CAMS, RIGS = 1280, 720, 4, 18
    K, D = synth.intrinsics(W, H)
    ext = synth.rig_extrinsics(CAMS)
    rng = np.random.default_rng(404)
    cams = []
    for r in range(RIGS):
        Twb = synth.random_base_pose(rng)
        for c in range(CAMS):
            Twc = Twb @ ext[c]
            cams.append(synth.make_cam(Twc[:3, :3], Twc[:3, 3], W, H))
    mb = M.Mantis(max_cams=RIGS * CAMS, max_width=W, max_height=H, iterations=iters)
    ms = M.Mantis(max_cams=CAMS, max_width=W, max_height=H, iterations=iters)
    try:
        assert RIGS * CAMS > M.lib().mantis_small_batch_frames(mb.h)
        for m in (mb, ms):
            m.set_map(*landmark_map)
            m.rng_state = 1
        fb = W * H * 3
        dev = mb.device_alloc(len(cams) * fb)
        mb.synth_render(cams, [synth.frame_seed(6, i) for i in range(len(cams))], dev)
        mb.synchronize()
        imgs = [M.make_image(None, K, D, T_base_cam=ext[i % CAMS], device_ptr=dev + i * fb, width=W, height=H)
                for i in range(len(cams))]
        rb, cb = mb.process(imgs, rigs=RIGS)
        dbg_b = [_debug_valid(mb.frame_debug(i)) for i in range(len(cams))]
        cnt_b = [mb.frame_counters(i)[:10].copy() for i in range(len(cams))]
        for r in range(RIGS):
            rs, cs = ms.process(imgs[r * CAMS:(r + 1) * CAMS], rigs=1)
            assert bytes(rs[0]) == bytes(rb[r]), f"rig {r}"
            for c in range(CAMS):
                assert bytes(cs[c]) == bytes(cb[r * CAMS + c]), f"rig {r} cam {c}"
                assert _debug_valid(ms.frame_debug(c)) == dbg_b[r * CAMS + c], f"rig {r} cam {c} debug record"
                a, b = ms.frame_counters(c)[:10], cnt_b[r * CAMS + c]
                assert np.array_equal(a[[0, 1, 2, 3, 4, 5, 6, 8, 9]], b[[0, 1, 2, 3, 4, 5, 6, 8, 9]]), (r, c)
        assert ms.rng_state == mb.rng_state
        mb.device_free(dev)
    finally:
        mb.close()
        ms.close()
