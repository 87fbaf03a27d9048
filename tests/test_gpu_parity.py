"""GPU parity: libmantis_amd.so (HIP, gfx950) against the CPU oracle.

Bar: bit-exact for integer/byte/index work (Canny, masks, quad corners,
projection counts, integer error sums => identical fast errors); poses from
identical decisions compared with an FP64 tolerance (1e-9 absolute) because
device libm (atan/sin/cos/tan/sqrt) may differ from glibc by an ulp.
"""
import os

import numpy as np
import pytest

import _oracle as O
from mantis_amd import synth

pytestmark = pytest.mark.gpu

POSE_TOL = 1e-9


@pytest.fixture(scope="module")
def mantis(landmark_map):
    import mantis_amd as M

    m = M.Mantis(max_cams=8, max_width=1280, max_height=720)
    m.set_map(*landmark_map)
    yield m
    m.close()


@pytest.fixture(scope="module")
def frames():
    rng = np.random.default_rng(1234)
    out = []
    for f in range(6):
        R, pos = synth.random_pose(rng)
        img = synth.render_host(synth.make_cam(R, pos), synth.frame_seed(2, f))
        out.append((img, R, pos))
    return out


def _img(frame):
    import mantis_amd as M

    K, D = synth.intrinsics()
    return M.make_image(frame[0], K, D)


def test_canny_bit_exact(mantis, frames):
    for fr in frames[:3]:
        got = mantis.canny(_img(fr))
        ref = O.canny(fr[0])
        assert np.array_equal(got, ref), f"canny differs at {np.argwhere(got != ref)[:10]}"


def test_canny_bit_exact_odd_sizes_and_noise(mantis):
    """Partial 128x32 tiles, W % 4 != 0 (byte-load path), seams crossed by
    long noisy components: smoothed noise gives dense, tangled candidates."""
    import mantis_amd as M

    rng = np.random.default_rng(77)
    K, D = synth.intrinsics()
    for (w, h) in [(907, 505), (1280, 720), (130, 35), (33, 7)]:
        base = rng.integers(0, 256, (h // 4 + 2, w // 4 + 2, 3)).astype(np.float64)
        img = np.repeat(np.repeat(base, 4, 0), 4, 1)[:h, :w]
        img = np.clip(img + rng.normal(0, 25, img.shape), 0, 255).astype(np.uint8)
        got = mantis.canny(M.make_image(img, K, D))
        ref = O.canny(img)
        assert np.array_equal(got, ref), f"{w}x{h}: canny differs at {np.argwhere(got != ref)[:10]}"


@pytest.mark.parametrize("strip", ["2", "1", "0"])
def test_canny_strip_and_tile_kernels_bit_exact(strip):
    """Both Canny kernels (k_canny_strip: column strips walked by one wave,
    DPP neighbour taps; k_canny: 128x32 LDS tiles; MANTIS_CANNY_STRIP picks)
    against the oracle on widths that end a strip mid-word, the first / last
    column groups at the frame edges, 3-row frames and blob noise."""
    import mantis_amd as M

    saved = os.environ.get("MANTIS_CANNY_STRIP")
    os.environ["MANTIS_CANNY_STRIP"] = strip
    try:
        mt = M.Mantis(max_cams=1, max_width=1280, max_height=720)
    finally:
        if saved is None:
            os.environ.pop("MANTIS_CANNY_STRIP")
        else:
            os.environ["MANTIS_CANNY_STRIP"] = saved
    rng = np.random.default_rng(5)
    K, D = synth.intrinsics()
    try:
        for (w, h) in [(1280, 720), (1000, 611), (232, 40), (448, 17), (8, 3), (224, 5), (12, 9)]:
            base = rng.integers(0, 256, (h // 3 + 2, w // 3 + 2, 3)).astype(np.float64)
            img = np.repeat(np.repeat(base, 3, 0), 3, 1)[:h, :w]
            img = np.clip(img + rng.normal(0, 30, img.shape), 0, 255).astype(np.uint8)
            got = mt.canny(M.make_image(img, K, D))
            ref = O.canny(img)
            assert np.array_equal(got, ref), f"{w}x{h}: canny differs at {np.argwhere(got != ref)[:10]}"
        # i.i.d. noise: more than 4096 candidate runs per 32-row band (the
        # hysteresis bands' global-label path)
        img = rng.integers(0, 256, (720, 1280, 3)).astype(np.uint8)
        got = mt.canny(M.make_image(img, K, D))
        ref = O.canny(img)
        assert np.array_equal(got, ref), f"noise: canny differs at {np.argwhere(got != ref)[:10]}"
    finally:
        mt.close()


def test_detector_binary_and_mask_bit_exact(mantis, frames):
    for fr in frames[:3]:
        det, mask = mantis.masks(_img(fr))
        cn = O.canny(fr[0])
        ref_det = O.detector_binary(cn)
        ref_mask = O.clean_mask(cn)
        assert np.array_equal(det, ref_det), f"detector binary differs: {np.count_nonzero(det != ref_det)} px"
        assert np.array_equal(mask, ref_mask), f"clean mask differs: {np.count_nonzero(mask != ref_mask)} px"


@pytest.mark.parametrize("walk,trace_lds", [("1048576", None), ("180", None), ("64", None), ("7", None), ("0", None),
                                             ("1048576", "0"), ("64", "0"), ("0", "0")])
def test_morphology_kernels_bit_exact(walk, trace_lds):
    """Both morphology kernels (k_morph_walk: one wave per frame row segment,
    stage windows in registers, MANTIS_MORPH_WALK = segment rows; with one
    segment per frame it also numbers the detector runs for the contour CCL;
    k_morph: LDS bands, MANTIS_MORPH_WALK=0) against the oracle's detector
    binary and cleanImageByEdge mask, and the contours that follow against
    findContours: widths ending mid-word, segments shorter than the 29-row
    reach, frames shorter than it, blob noise and i.i.d. noise. With
    MANTIS_TRACE_LDS_FRAMES=0 the borders are walked on the tiled plane in L2
    (k_tile_bits' 16-pixel-group windows of three rows)."""
    import mantis_amd as M

    env = {"MANTIS_MORPH_WALK": walk}
    if trace_lds is not None:  # the L2 walker on the tiled plane
        env["MANTIS_TRACE_LDS_FRAMES"] = trace_lds
    saved = {k: os.environ.get(k) for k in env}
    os.environ.update(env)
    try:
        mt = M.Mantis(max_cams=1, max_width=1920, max_height=1080, max_contour_points=1 << 21)
    finally:
        for k, v in saved.items():
            if v is None:
                os.environ.pop(k)
            else:
                os.environ[k] = v
    rng = np.random.default_rng(17)
    K, D = synth.intrinsics()
    try:
        sizes = [(1280, 720), (1920, 1080), (1000, 611), (232, 40), (33, 7), (64, 30), (95, 61)]
        for k, (w, h) in enumerate(sizes):
            if k % 2 == 0:
                base = rng.integers(0, 256, (h // 5 + 2, w // 5 + 2, 3)).astype(np.float64)
                img = np.repeat(np.repeat(base, 5, 0), 5, 1)[:h, :w]
                img = np.clip(img + rng.normal(0, 30, img.shape), 0, 255).astype(np.uint8)
            else:
                img = rng.integers(0, 256, (h, w, 3)).astype(np.uint8)
            det, mask = mt.masks(M.make_image(img, K, D))
            cn = O.canny(img)
            ref_det = O.detector_binary(cn)
            ref_mask = O.clean_mask(cn)
            assert np.array_equal(det, ref_det), f"{w}x{h}: detector binary differs: {np.count_nonzero(det != ref_det)} px"
            assert np.array_equal(mask, ref_mask), f"{w}x{h}: clean mask differs: {np.count_nonzero(mask != ref_mask)} px"
            if k % 2 == 1 and w * h > 100000:
                continue  # i.i.d. noise at full size: masks only (its contours are millions of points)
            mt.detect_quads(M.make_image(img, K, D))
            cnt = mt.frame_counters(0)
            cs, _ = O.find_contours(ref_det, 2)
            assert cnt[8] == 0, f"{w}x{h}: overflow flags {cnt[8]}"
            assert cnt[0] == len(cs), f"{w}x{h}: borders {cnt[0]} vs findContours {len(cs)}"
            _contours_equal(mt, img)
    finally:
        mt.close()


def test_quads_bit_exact(mantis, frames, landmark_map):
    orc = O.Oracle(*landmark_map)
    K, D = synth.intrinsics()
    for fr in frames[:3]:
        got = mantis.detect_quads(_img(fr))
        dbg = orc.process(fr[0], K, D)
        ref = np.array(dbg.quads)[: dbg.n_quads]
        assert got.shape == ref.shape, f"quad count {len(got)} vs oracle {len(ref)}"
        assert np.array_equal(got, ref)


def test_contour_borders_match_find_contours(mantis, frames):
    """Run-length CCL + parallel border following against findContours(CCOMP,
    SIMPLE) on the detector binary: same number of borders (outer + hole) and
    the same total of chain points, on real frames and on blob-noise images
    with many nested components and holes."""
    import mantis_amd as M

    K, D = synth.intrinsics()
    rng = np.random.default_rng(99)
    imgs = [fr[0] for fr in frames[:2]]
    for (w, h, cell) in [(1280, 720, 6), (640, 480, 3), (333, 97, 2)]:
        base = (rng.random((h // cell + 2, w // cell + 2)) > 0.5).astype(np.float64) * 200 + 20
        img = np.repeat(np.repeat(base, cell, 0), cell, 1)[:h, :w]
        imgs.append(np.repeat(img[:, :, None], 3, 2).astype(np.uint8))
    for img in imgs:
        mantis.detect_quads(M.make_image(img, K, D))
        cnt = mantis.frame_counters(0)
        cs, holes = O.find_contours(O.detector_binary(O.canny(img)), 2)
        assert cnt[8] == 0, f"overflow flags {cnt[8]}"
        assert cnt[0] == len(cs), f"borders {cnt[0]} vs findContours {len(cs)}"
        assert cnt[1] == sum(len(c) for c in cs), f"points {cnt[1]} vs {sum(len(c) for c in cs)}"
        _contours_equal(mantis, img)


def _contours_equal(mt, img):
    """Every border's point sequence from the library equals one of
    findContours' (CCOMP, SIMPLE) exactly, start point and order included,
    as a multiset over the frame."""
    import collections

    got = collections.Counter((h, tuple(map(tuple, p))) for p, h in mt.contours(0))
    cs, holes = O.find_contours(O.detector_binary(O.canny(img)), 2)
    want = collections.Counter((h, tuple(map(tuple, np.asarray(c).reshape(-1, 2)))) for c, h in zip(cs, holes))
    assert got == want, f"{sum((got - want).values())} borders differ of {len(cs)}"


@pytest.mark.parametrize("seg_m", ["0", "32", "8"])
def test_segmented_border_walks_point_sequences(frames, seg_m):
    """Border walks split at checkpoints (k_seg_plan: the visits of foreground
    run ends in rows y = M k; MANTIS_SEG_M, 0 = whole borders) on the
    large-batch walker: each border's chain points equal findContours' point
    for point, on real frames and on blob-noise images with many nested
    components, holes and one-pixel runs (a 16-point chunk per segment's
    tail stays within the point pool)."""
    import os

    import mantis_amd as M

    K, D = synth.intrinsics()
    rng = np.random.default_rng(77)
    imgs = [fr[0] for fr in frames[:2]]
    for (w, h, cell) in [(1280, 720, 6), (640, 480, 1), (333, 97, 2)]:
        base = (rng.random((h // cell + 2, w // cell + 2)) > 0.5).astype(np.float64) * 200 + 20
        img = np.repeat(np.repeat(base, cell, 0), cell, 1)[:h, :w]
        imgs.append(np.repeat(img[:, :, None], 3, 2).astype(np.uint8))
    saved = {k: os.environ.get(k) for k in ("MANTIS_TRACE_LDS_FRAMES", "MANTIS_SEG_M")}
    os.environ["MANTIS_TRACE_LDS_FRAMES"] = "0"
    os.environ["MANTIS_SEG_M"] = seg_m
    try:
        mt = M.Mantis(max_cams=1, max_width=1280, max_height=720)
    finally:
        for k, v in saved.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
    try:
        for img in imgs:
            try:
                mt.detect_quads(M.make_image(img, K, D))
            except M.MantisError:
                pass  # the dense one-pixel noise can exceed the point pool; checked below
            cnt = mt.frame_counters(0)
            if cnt[8]:
                assert img.shape[:2] == (480, 640), f"overflow flags {cnt[8]}"
                continue
            if seg_m != "0" and img.shape[:2] == (720, 1280):
                assert cnt[22] > 0 and cnt[23] == int(seg_m), "frame walked unsplit"
            _contours_equal(mt, img)
    finally:
        mt.close()


def test_throughput_border_walks_match_find_contours(landmark_map):
    """The large-batch border walker (one wave per frame refilled from the
    border list, 64-bit row windows in 32-row tiles) forced on single frames
    (MANTIS_TRACE_LDS_FRAMES=0): borders and chain points against
    findContours on blob-noise images whose padded sizes are not multiples of
    32 (partial tiles, partial CCL bands) and on a real frame."""
    import os

    import mantis_amd as M

    K, D = synth.intrinsics()
    rng = np.random.default_rng(123)
    imgs = []
    for (w, h, cell) in [(333, 97, 2), (1000, 611, 6), (640, 480, 3), (1280, 720, 6)]:
        base = (rng.random((h // cell + 2, w // cell + 2)) > 0.5).astype(np.float64) * 200 + 20
        img = np.repeat(np.repeat(base, cell, 0), cell, 1)[:h, :w]
        imgs.append(np.repeat(img[:, :, None], 3, 2).astype(np.uint8))
    old = os.environ.get("MANTIS_TRACE_LDS_FRAMES")
    os.environ["MANTIS_TRACE_LDS_FRAMES"] = "0"
    try:
        mt = M.Mantis(max_cams=2, max_width=1280, max_height=720)
    finally:
        if old is None:
            del os.environ["MANTIS_TRACE_LDS_FRAMES"]
        else:
            os.environ["MANTIS_TRACE_LDS_FRAMES"] = old
    try:
        for img in imgs:
            mt.detect_quads(M.make_image(img, K, D))
            cnt = mt.frame_counters(0)
            cs, holes = O.find_contours(O.detector_binary(O.canny(img)), 2)
            assert cnt[8] == 0, f"overflow flags {cnt[8]}"
            assert cnt[0] == len(cs), f"borders {cnt[0]} vs findContours {len(cs)}"
            assert cnt[1] == sum(len(c) for c in cs), f"points {cnt[1]} vs {sum(len(c) for c in cs)}"
    finally:
        mt.close()


def test_rpp_batch_matches_oracle(mantis):
    rng = np.random.default_rng(7)
    s = 0.16
    sq = [np.array([[s, -s, -s, s], [s, s, -s, -s], [0, 0, 0, 0.0]]),
          np.array([[s, -s, -s, s], [-s, -s, s, s], [0, 0, 0, 0.0]])]
    img_pts, obj_pts, refs = [], [], []
    for k in range(256):
        R = synth.rot_z(rng.uniform(0, 6.28)) @ synth.NADIR @ synth.rot_x(rng.normal() * 0.3)
        t = np.array([rng.normal() * 0.3, rng.normal() * 0.3, rng.uniform(0.8, 3)])
        m = sq[k % 2]
        Q = R.T @ m + t[:, None]
        ip = np.vstack([Q[0] / Q[2], Q[1] / Q[2], np.ones(4)])
        ip[:2] += rng.normal(size=(2, 4)) * 0.003
        img_pts.append(ip[:2].T.copy())
        obj_pts.append(m.T.copy())
        refs.append(O.rpp(m, ip))
    R, t, e, st = mantis.rpp(np.array(img_pts), np.array(obj_pts))
    for k, (rs, rR, rt, re, _) in enumerate(refs):
        assert st[k] == rs
        np.testing.assert_allclose(R[k], rR, atol=POSE_TOL, rtol=0)
        np.testing.assert_allclose(t[k], rt, atol=POSE_TOL, rtol=0)
        np.testing.assert_allclose(e[k], re[:2], rtol=1e-9, atol=1e-15)


def test_rpp_demo_known_answer_on_gpu(mantis):
    """The reference's only known answer on the hot path, run by the device
    RPP: demo.cpp:17-38's 10-point problem (mantis_rpp_solve, mk_rpp.h's
    functions instantiated for 10 points) against demo.cpp's Matlab R, t
    (printed to 5 decimals: 1e-4 + half a printed unit) and against the oracle."""
    d = np.load(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "rpp_demo.npz"),
                allow_pickle=False)
    R, t, e, st, it = mantis.rpp_solve(d["model"], d["iprts"])
    assert st[0] == 1
    np.testing.assert_allclose(R[0], d["matlab_R"], atol=1e-4 + 5e-6, rtol=0)
    np.testing.assert_allclose(t[0], d["matlab_t"], atol=1e-4 + 5e-6, rtol=0)
    ost, oR, ot, oe, code = O.rpp(d["model"], d["iprts"])
    assert ost == 1 and code == 0
    np.testing.assert_allclose(R[0], oR, atol=POSE_TOL, rtol=0)
    np.testing.assert_allclose(t[0], ot, atol=POSE_TOL, rtol=0)
    np.testing.assert_allclose(e[0], oe[:2], rtol=1e-9, atol=1e-15)
    assert it[0] == int(oe[2])
    # the committed fixture is the oracle's output for this problem
    np.testing.assert_allclose(R[0], d["R"], atol=POSE_TOL, rtol=0)


@pytest.mark.parametrize("npts", [4, 5, 7, 10, 12])
def test_rpp_solve_n_points_matches_oracle(mantis, npts):
    """mantis_rpp_solve on random planar n-point problems (noisy projections of
    a random plane patch) against the oracle's RPP::Rpp restatement; n = 4 also
    against mantis_rpp_batch (the queue path runs the same functions)."""
    rng = np.random.default_rng(100 + npts)
    models, iprts, refs = [], [], []
    for k in range(48):
        m = np.vstack([rng.uniform(-0.8, 0.8, size=(2, npts)), np.zeros((1, npts))])
        R0 = synth.rot_z(rng.uniform(0, 6.28)) @ synth.NADIR @ synth.rot_x(rng.normal() * 0.4)
        t0 = np.array([rng.normal() * 0.3, rng.normal() * 0.3, rng.uniform(2, 12)])
        Q = R0.T @ m + t0[:, None]
        ip = np.vstack([Q[0] / Q[2], Q[1] / Q[2], np.ones(npts)])
        ip[:2] += rng.normal(size=(2, npts)) * 0.002
        models.append(m)
        iprts.append(ip)
        refs.append(O.rpp(m, ip))
    R, t, e, st, it = mantis.rpp_solve(np.array(models), np.array(iprts))
    for k, (rs, rR, rt, re, code) in enumerate(refs):
        assert st[k] == (-1 if code == 1 else rs), k
        np.testing.assert_allclose(R[k], rR, atol=POSE_TOL, rtol=0)
        np.testing.assert_allclose(t[k], rt, atol=POSE_TOL * max(1.0, np.abs(rt).max()), rtol=0)
        np.testing.assert_allclose(e[k], re[:2], rtol=1e-9, atol=1e-15)
        assert it[k] == int(re[2]), k
    if npts == 4:
        img = np.array([ip[:2].T for ip in iprts])
        obj = np.array([m.T for m in models])
        Rb, tb, eb, sb = mantis.rpp(img, obj)
        assert np.array_equal(Rb, R) and np.array_equal(tb, t) and np.array_equal(eb, e) and np.array_equal(sb, st)


def test_rpp_solve_rejects_bad_point_counts(mantis):
    import mantis_amd as M

    m = np.zeros((3, 13))
    q = np.ones((3, 13))
    with pytest.raises(M.MantisError):
        mantis.rpp_solve(m, q)


def test_scoring_matches_oracle(mantis, frames, landmark_map):
    orc = O.Oracle(*landmark_map)
    K, D = synth.intrinsics()
    rng = np.random.default_rng(3)
    for fr in frames[:2]:
        img, R, pos = fr
        base = synth.truth_c2w(R, pos)
        c2w = [base]
        for _ in range(255):
            Rp = synth.rot_x(rng.normal() * 0.03) @ synth.rot_y(rng.normal() * 0.03) @ synth.rot_z(rng.normal() * 0.03)
            Rw = R @ Rp
            c2w.append(synth.truth_c2w(Rw, pos + rng.normal(size=3) * 0.01))
        c2w = np.array(c2w)
        for fast in (True, False):
            ge, gn = mantis.score(_img(fr), c2w, fast=fast)
            oe, on = orc.score(img, K, D, c2w, fast=fast)
            assert np.array_equal(gn, on)
            if fast:
                assert np.array_equal(ge, oe), "fast errors are integer sums / (n*1.1): must be identical"
            else:
                np.testing.assert_allclose(ge, oe, rtol=1e-13)


def _cmp_debug(g, o, label):
    assert g.reason == o.reason, f"{label}: reason {g.reason} vs {o.reason}"
    assert g.n_raw_quads == o.n_raw_quads, f"{label}: raw quads {g.n_raw_quads} vs {o.n_raw_quads}"
    assert g.n_quads == o.n_quads
    n = g.n_quads
    assert np.array_equal(np.array(g.quads)[:n], np.array(o.quads)[:n])
    np.testing.assert_allclose(np.array(g.test_pts)[:n], np.array(o.test_pts)[:n], atol=1e-12, rtol=0)
    assert g.n_gen == o.n_gen, f"{label}: generated hyps {g.n_gen} vs {o.n_gen}"
    assert g.n_hyps == o.n_hyps, f"{label}: clustered hyps {g.n_hyps} vs {o.n_hyps}"
    if o.reason in (1, 2):
        return
    c = g.n_hyps
    np.testing.assert_allclose(np.array(g.hyp_c2w)[:c], np.array(o.hyp_c2w)[:c], atol=POSE_TOL, rtol=0)
    assert np.array_equal(np.array(g.hyp_n)[:c], np.array(o.hyp_n)[:c])
    assert np.array_equal(np.array(g.hyp_err)[:c], np.array(o.hyp_err)[:c])
    assert g.best1_err == o.best1_err
    np.testing.assert_array_equal(np.array(g.pf_iter_err), np.array(o.pf_iter_err))
    np.testing.assert_allclose(np.array(g.pf_c2w), np.array(o.pf_c2w), atol=POSE_TOL, rtol=0)
    np.testing.assert_array_equal(np.array(g.shift_err), np.array(o.shift_err))
    np.testing.assert_array_equal(np.array(g.top20_err), np.array(o.top20_err))
    np.testing.assert_allclose(np.array(g.yaw_err), np.array(o.yaw_err), rtol=1e-12)
    assert g.yaw_best == o.yaw_best
    assert g.publish == o.publish
    np.testing.assert_allclose(np.array(g.position), np.array(o.position), atol=POSE_TOL, rtol=0)
    np.testing.assert_allclose(np.array(g.orientation_xyzw), np.array(o.orientation_xyzw), atol=POSE_TOL, rtol=0)
    np.testing.assert_allclose(g.pub_error, o.pub_error, rtol=1e-12)


def test_full_pipeline_matches_oracle(mantis, frames, landmark_map):
    """Whole callback on a batch of frames; RNG stream shared across frames."""
    orc = O.Oracle(*landmark_map, seed=1)
    K, D = synth.intrinsics()
    mantis.rng_state = 1
    imgs = [_img(fr) for fr in frames]
    rig, cams = mantis.process(imgs, rigs=len(imgs))
    for i, fr in enumerate(frames):
        o = orc.process(fr[0], K, D)
        g = mantis.frame_debug(i)
        _cmp_debug(g, o, f"frame {i}")
        assert cams[i].reason == o.reason
        assert cams[i].publish == o.publish
    assert mantis.rng_state == orc.rng_state, "cv::RNG stream must advance exactly as the reference's"


def test_small_batch_objpose_queue_settings(frames, landmark_map):
    """The rig-latency ObjPose queues (k_objpose_q: RPP.cpp:66-208's ObjPose as a
    job queue) at every public setting of MANTIS_OP_LANES_SMALL (jobs per wave)
    x MANTIS_OP_ROUNDS_SMALL (tail-compaction rounds): one 4-camera rig, every
    camera result and frame record byte-identical to the default context's, and
    the one-job-per-wave single-round setting against the oracle. Round 4's
    job-duplication failure (non-reserved lanes took jobs) lived on this path."""
    import mantis_amd as M

    K, D = synth.intrinsics()
    imgs = [M.make_image(fr[0], K, D) for fr in frames[:4]]

    def run(env):
        saved = {k: os.environ.get(k) for k in env}
        os.environ.update(env)
        try:
            m = M.Mantis(max_cams=4, max_width=1280, max_height=720)
        finally:
            for k, v in saved.items():
                if v is None:
                    os.environ.pop(k)
                else:
                    os.environ[k] = v
        try:
            assert M.lib().mantis_small_batch_frames(m.h) >= 4
            m.set_map(*landmark_map)
            m.rng_state = 1
            rig, cams = m.process(imgs, rigs=1)
            return (bytes(rig[0]), [bytes(c) for c in cams], [bytes(m.frame_debug(f)) for f in range(4)],
                    m.rng_state, [m.frame_debug(f) for f in range(4)])
        finally:
            m.close()

    ref = run({})
    for lanes in ("1", "4", "64"):
        for rounds in ("1", "6"):
            got = run({"MANTIS_OP_LANES_SMALL": lanes, "MANTIS_OP_ROUNDS_SMALL": rounds})
            tag = f"lanes {lanes} rounds {rounds}"
            assert got[0] == ref[0], f"{tag}: rig result differs"
            for f in range(4):
                assert got[1][f] == ref[1][f], f"{tag}: camera {f} result differs"
                assert got[2][f] == ref[2][f], f"{tag}: camera {f} frame record differs"
            assert got[3] == ref[3], f"{tag}: cv::RNG state differs"
            if lanes == "1" and rounds == "1":
                orc = O.Oracle(*landmark_map, seed=1)
                for f, fr in enumerate(frames[:4]):
                    _cmp_debug(got[4][f], orc.process(fr[0], K, D), f"{tag} frame {f}")


def test_throughput_mode_kernels_match_latency_mode(frames, landmark_map):
    """Large batches take other kernel shapes (border walks from L2 instead of an
    LDS copy of the bit plane, 256-thread contour blocks): force them on a small
    batch (MANTIS_TRACE_LDS_FRAMES=0) and compare everything against the
    latency-mode context (itself checked against the oracle above)."""
    import os

    import mantis_amd as M

    K, D = synth.intrinsics()
    imgs = [M.make_image(fr[0], K, D) for fr in frames[:4]]
    old = os.environ.get("MANTIS_TRACE_LDS_FRAMES")
    os.environ["MANTIS_TRACE_LDS_FRAMES"] = "0"
    try:
        mt = M.Mantis(max_cams=4, max_width=1280, max_height=720)
    finally:
        if old is None:
            del os.environ["MANTIS_TRACE_LDS_FRAMES"]
        else:
            os.environ["MANTIS_TRACE_LDS_FRAMES"] = old
    ml = M.Mantis(max_cams=4, max_width=1280, max_height=720)
    try:
        for m in (mt, ml):
            m.set_map(*landmark_map)
            m.rng_state = 1
        _, ct = mt.process(imgs)
        _, cl = ml.process(imgs)
        for f in range(len(imgs)):
            gt, gl = mt.frame_debug(f), ml.frame_debug(f)
            assert list(mt.frame_counters(f)[:2]) == list(ml.frame_counters(f)[:2])  # borders, points
            assert gt.n_quads == gl.n_quads and gt.n_quads > 0
            n = gt.n_quads
            assert np.array_equal(np.array(gt.quads)[:n], np.array(gl.quads)[:n])
            assert gt.pf_err == gl.pf_err and gt.n_hyps == gl.n_hyps
            assert ct[f].reason == cl[f].reason and ct[f].publish == cl[f].publish
            assert list(ct[f].position) == list(cl[f].position)
        assert mt.rng_state == ml.rng_state
    finally:
        mt.close()
        ml.close()


def test_mixed_batch_skipped_frames_keep_rng_stream(mantis, frames, landmark_map):
    """Frames that return early (no quadrilaterals: a flat frame, a noise-only
    frame; the reference's early returns, src/mantis3.cpp:82-84) draw no
    gaussians, so the particle filters of the later frames in the same batch
    read the stream from the same position as the sequential reference does
    (device prefix over the frames that reach the particle filter). Also a
    frame with a ragged width (row stride > 3 W)."""
    import mantis_amd as M

    K, D = synth.intrinsics()
    flat = np.full((720, 1280, 3), 90, np.uint8)
    rng = np.random.default_rng(4)
    noise = rng.integers(80, 120, (720, 1280, 3), dtype=np.uint8)
    seq = [frames[0][0], flat, frames[1][0], noise, frames[2][0], flat]
    orc = O.Oracle(*landmark_map, seed=1)
    mantis.rng_state = 1
    imgs = []
    for k, img in enumerate(seq):
        if k == 2:  # padded rows: step = 3 W + 48
            padded = np.zeros((720, 3 * 1280 + 48), np.uint8)
            padded[:, :3 * 1280] = img.reshape(720, -1)
            im = M.make_image(img, K, D)
            keep = padded
            im.bgr = keep.ctypes.data
            im.step_bytes = 3 * 1280 + 48
            imgs.append((im, keep))
        else:
            imgs.append((M.make_image(img, K, D), None))
    rig, cams = mantis.process([im for im, _ in imgs], rigs=len(imgs))
    for i, img in enumerate(seq):
        o = orc.process(img, K, D)
        assert cams[i].reason == o.reason, f"frame {i}: reason {cams[i].reason} vs {o.reason}"
        assert cams[i].publish == o.publish
        if o.reason != 1:  # frames with quads: same decisions and pose as the reference
            _cmp_debug(mantis.frame_debug(i), o, f"frame {i}")
    assert cams[1].reason == 1 and cams[5].reason == 1, "flat frames have no quadrilaterals"
    assert mantis.rng_state == orc.rng_state


def test_odd_capacity_multi_frame_batch(landmark_map):
    """A context whose padded plane (max_width + 2) x (max_height + 2) is not a
    multiple of 4 bytes (1283 x 723), with several frames per batch: the
    hysteresis flag plane of frame f >= 1 must stay dword-aligned for its
    32-bit flag atomics. Frames of an odd size (1279 x 719) go
    through the whole callback and match the oracle frame by frame."""
    import mantis_amd as M

    W, H = 1279, 719
    K, D = synth.intrinsics(W, H)
    rng = np.random.default_rng(55)
    m = M.Mantis(max_cams=3, max_width=1281, max_height=721)
    try:
        m.set_map(*landmark_map)
        m.rng_state = 1
        seq = []
        for f in range(3):
            R, pos = synth.random_pose(rng)
            seq.append(synth.render_host(synth.make_cam(R, pos, W, H), synth.frame_seed(7, f)))
        _, cams = m.process([M.make_image(img, K, D) for img in seq], rigs=3)
        orc = O.Oracle(*landmark_map, seed=1)
        for i, img in enumerate(seq):
            o = orc.process(img, K, D)
            assert o.n_quads > 0
            _cmp_debug(m.frame_debug(i), o, f"odd frame {i}")
            assert cams[i].reason == o.reason and cams[i].publish == o.publish
        assert m.rng_state == orc.rng_state
    finally:
        m.close()


def test_screen_off_equals_screen_on(frames, landmark_map):
    """The fast scorers' FP32 projection screen (mk_screen.h) against the
    exact FP64 path: a context created with MANTIS_SCREEN=0 sends every
    landmark through the exact fallback (the block queues overflow, so the
    in-place path runs too, then the drains); every error, count and decision
    must be identical, in the pipeline (init / particle filter / shifts) and in
    the standalone scorer (k_score_api, with and without a mask)."""
    import os

    import mantis_amd as M

    K, D = synth.intrinsics()
    imgs = [M.make_image(fr[0], K, D) for fr in frames[:4]]
    old = os.environ.get("MANTIS_SCREEN")
    os.environ["MANTIS_SCREEN"] = "0"
    try:
        mx = M.Mantis(max_cams=4, max_width=1280, max_height=720)
    finally:
        if old is None:
            del os.environ["MANTIS_SCREEN"]
        else:
            os.environ["MANTIS_SCREEN"] = old
    ms = M.Mantis(max_cams=4, max_width=1280, max_height=720)
    try:
        for m in (mx, ms):
            m.set_map(*landmark_map)
            m.rng_state = 1
        _, cx = mx.process(imgs)
        _, cs = ms.process(imgs)
        for f in range(len(imgs)):
            gx, gs = mx.frame_debug(f), ms.frame_debug(f)
            assert gx.n_hyps == gs.n_hyps and gx.n_hyps > 0
            c = gx.n_hyps
            assert np.array_equal(np.array(gx.hyp_err)[:c], np.array(gs.hyp_err)[:c])
            assert np.array_equal(np.array(gx.hyp_n)[:c], np.array(gs.hyp_n)[:c])
            assert np.array_equal(np.array(gx.pf_iter_err), np.array(gs.pf_iter_err))
            assert np.array_equal(np.array(gx.shift_err), np.array(gs.shift_err))
            assert np.array_equal(np.array(gx.top20_err), np.array(gs.top20_err))
            assert gx.yaw_best == gs.yaw_best and gx.publish == gs.publish
            assert list(cx[f].position) == list(cs[f].position)
        assert mx.rng_state == ms.rng_state
        rng = np.random.default_rng(5)
        img, R, pos = frames[0]
        c2w = [synth.truth_c2w(R @ synth.rot_z(rng.normal() * 0.05), pos + rng.normal(size=3) * 0.02)
               for _ in range(300)]
        c2w = np.array(c2w)
        for mask in (None, ms.masks(imgs[0])[1]):
            ex, nx = mx.score(imgs[0], c2w, fast=True, mask=mask)
            es, ns = ms.score(imgs[0], c2w, fast=True, mask=mask)
            assert np.array_equal(nx, ns) and np.array_equal(ex, es)
    finally:
        mx.close()
        ms.close()


def _disc_frame(rows, cols, pitch=26, r=5, squares=True):
    """Gray frame with a rows x cols lattice of dark discs (each becomes a
    small hole of the dilated edge net: a border whose approxPolyDP is not a
    quad) and, when `squares`, three large dark squares on the right (quads)."""
    H, W = 720, 1280
    img = np.full((H, W, 3), 200, np.uint8)
    yy, xx = np.mgrid[0:H, 0:W]
    for i in range(rows):
        for j in range(cols):
            cy, cx = 20 + pitch * i, 20 + pitch * j
            img[(yy - cy) ** 2 + (xx - cx) ** 2 <= r * r] = 40
    if squares:
        for k, (y0, x0) in enumerate([(60, 1000), (300, 1060), (520, 980)]):
            img[y0:y0 + 110 + 10 * k, x0:x0 + 120] = 30
    return img


@pytest.mark.parametrize("lds_frames", [None, "0"])
def test_many_borders_approx_paths(landmark_map, lds_frames):
    """k_frame_contours' approxPolyDP on frames with 906 and 2,366 borders:
    the length-ordered path (<= 1024 borders) and the index-order fallback
    (more), in the latency shape (1024-thread blocks, LDS walks) and, with
    MANTIS_TRACE_LDS_FRAMES=0, the throughput shape (256-thread blocks, L2
    walks): quads, raw quad count and border / point counts against the oracle."""
    import mantis_amd as M

    K, D = synth.intrinsics()
    seq = [_disc_frame(18, 25), _disc_frame(30, 40, pitch=24)]  # 906 / 2,366 borders
    old = os.environ.get("MANTIS_TRACE_LDS_FRAMES")
    if lds_frames is not None:
        os.environ["MANTIS_TRACE_LDS_FRAMES"] = lds_frames
    try:
        m = M.Mantis(max_cams=2, max_width=1280, max_height=720)
    finally:
        if old is None:
            os.environ.pop("MANTIS_TRACE_LDS_FRAMES", None)
        else:
            os.environ["MANTIS_TRACE_LDS_FRAMES"] = old
    try:
        m.set_map(*landmark_map)
        m.rng_state = 1
        m.process([M.make_image(x, K, D) for x in seq], rigs=2)
        orc = O.Oracle(*landmark_map, seed=1)
        nbs = []
        for i, x in enumerate(seq):
            o = orc.process(x, K, D)
            g = m.frame_debug(i)
            nbs.append(int(m.frame_counters(i)[0]))
            assert g.n_raw_quads == o.n_raw_quads and g.n_quads == o.n_quads and o.n_quads > 0, (i, g.n_quads, o.n_quads)
            n = g.n_quads
            assert np.array_equal(np.array(g.quads)[:n], np.array(o.quads)[:n]), i
        assert nbs[0] <= 1024 < nbs[1], nbs  # both approx paths ran
    finally:
        m.close()
