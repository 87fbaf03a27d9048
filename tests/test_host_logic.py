"""Device-logic headers (mantis_amd/csrc/mk_*.h) compiled for the host
(build/libmantis_hostcheck.so) against the oracle and the goldens, on CPU.

These are the exact per-work-item algorithms the HIP kernels run (RPP phases,
Jenkins-Traub, libstdc++ sort port, border following, approxPolyDP, the
parallel contour formulation, bit-packed morphology, fisheye maps), so a
mismatch here is a device bug found without a GPU. Bar: bit-exact.
"""
import os

import numpy as np
import pytest

import _hostcheck as H
import _oracle as O
from mantis_amd import synth

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def test_rpp_phases_vs_reference_golden():
    d = np.load(os.path.join(GOLD, "rpp_golden.npz"), allow_pickle=False)
    for k in range(len(d["model"])):
        st, R, t, e, code = H.rpp(d["model"][k], d["iprts"][k])
        assert st == d["status"][k], d["name"][k]
        assert np.array_equal(R.reshape(-1), d["R"][k].reshape(-1)), d["name"][k]
        assert np.array_equal(t, d["t"][k]) and np.array_equal(e, d["errs"][k]), d["name"][k]


def test_rpp_phases_vs_oracle_hard_cases():
    rng = np.random.default_rng(77)
    s = 0.16
    sq = [np.array([[s, -s, -s, s], [s, s, -s, -s], [0, 0, 0, 0.0]]),
          np.array([[s, -s, -s, s], [-s, -s, s, s], [0, 0, 0, 0.0]])]
    for k in range(600):
        R = synth.rot_z(rng.uniform(0, 6.3)) @ synth.NADIR @ synth.rot_x(rng.normal() * 1.5)
        t = np.array([rng.normal() * 0.3, rng.normal() * 0.3, rng.uniform(0.5, 3)])
        m = sq[k % 2]
        Q = R.T @ m + t[:, None]
        ip = np.vstack([Q[0] / Q[2], Q[1] / Q[2], np.ones(4)])
        ip[:2] += rng.normal(size=(2, 4)) * 0.05
        a, b = H.rpp(m, ip), O.rpp(m, ip)
        assert a[0] == b[0] and a[4] == b[4]
        for u, v in zip(a[1:4], b[1:4]):
            assert np.array_equal(u, v, equal_nan=True)


def test_rpp_n_points_host_build_vs_oracle():
    """mantis_rpp_solve's per-point-count instances (mk_rpp_np.inc), host
    build, bit-exact against the oracle's RPP on demo.cpp's 10-point problem
    and on random planar problems of 4..12 points."""
    d = np.load(os.path.join(GOLD, "rpp_demo.npz"), allow_pickle=False)
    a, b = H.rpp_n(d["model"], d["iprts"]), O.rpp(d["model"], d["iprts"])
    assert a[0] == b[0] == 1 and a[4] == b[4] == 0
    for u, v in zip(a[1:4], b[1:4]):
        assert np.array_equal(u, v)
    np.testing.assert_allclose(a[1], d["matlab_R"], atol=1e-4 + 5e-6, rtol=0)
    np.testing.assert_allclose(a[2], d["matlab_t"], atol=1e-4 + 5e-6, rtol=0)
    rng = np.random.default_rng(5)
    for n in range(4, 13):
        for k in range(40):
            m = np.vstack([rng.uniform(-0.8, 0.8, size=(2, n)), np.zeros((1, n))])
            R = synth.rot_z(rng.uniform(0, 6.3)) @ synth.NADIR @ synth.rot_x(rng.normal() * 0.6)
            t = np.array([rng.normal() * 0.3, rng.normal() * 0.3, rng.uniform(1, 12)])
            Q = R.T @ m + t[:, None]
            ip = np.vstack([Q[0] / Q[2], Q[1] / Q[2], np.ones(n)])
            ip[:2] += rng.normal(size=(2, n)) * 0.01
            a, b = H.rpp_n(m, ip), O.rpp(m, ip)
            assert a[0] == b[0] and a[4] == b[4], (n, k)
            for u, v in zip(a[1:4], b[1:4]):
                assert np.array_equal(u, v, equal_nan=True), (n, k)


def test_jacobi_noise_fast_forward_is_bit_exact():
    """mk_rpp.h jacobi_noise_ff skips the Jacobi sweeps that only shrink the
    rank-deficient row of a planar problem; every output byte (signs of zero
    included) must equal the full sweep sequence, on realistic, adversarial
    (scales 1e-3..1e2, noise 1e-6..0.3, rounded image points) and degenerate
    (repeated / collinear points) problems."""
    rng = np.random.default_rng(2024)
    try:
        for k in range(3000):
            s = 10 ** rng.uniform(-3, 2) if k % 2 else 0.16
            m = np.array([[s, -s, -s, s], [s, s, -s, -s], [0, 0, 0, 0.0]])
            if k % 4 == 1:
                m[1] = -m[1]
            if k % 4 == 2:
                m = np.vstack([rng.uniform(-s, s, size=(2, 4)), np.zeros((1, 4))])
            if k % 13 == 0:
                m[:, 3] = m[:, 2]
            if k % 17 == 0:
                m[1] = m[0] * 0.5
            R = synth.rot_z(rng.uniform(0, 6.3)) @ synth.NADIR @ synth.rot_x(rng.normal() * 1.2)
            t = np.array([rng.normal() * 2 * s, rng.normal() * 2 * s, rng.uniform(1.5, 90) * s])
            Q = R.T @ m + t[:, None]
            ip = np.vstack([Q[0] / Q[2], Q[1] / Q[2], np.ones(4)])
            ip[:2] += rng.normal(size=(2, 4)) * 10 ** rng.uniform(-6, -0.5)
            if k % 7 == 0:
                ip[:2] = np.round(ip[:2] * 64) / 64
            H.set_jacobi_ff(False)
            a = H.rpp(m, ip)
            H.set_jacobi_ff(True)
            b = H.rpp(m, ip)
            assert a[0] == b[0] and a[4] == b[4], k
            for u, v in zip(a[1:4], b[1:4]):
                assert u.tobytes() == v.tobytes(), k
    finally:
        H.set_jacobi_ff(True)


def test_rpoly_vs_reference_golden():
    d = np.load(os.path.join(GOLD, "rpoly_golden.npz"), allow_pickle=False)
    for k in range(len(d["coef"])):
        deg, zr, zi = H.rpoly(d["coef"][k])
        assert deg == d["degree"][k]
        assert np.array_equal(zr, d["zr"][k]) and np.array_equal(zi, d["zi"][k])


def test_sort_desc_matches_libstdcxx():
    rng = np.random.default_rng(5)
    for n in (1, 2, 15, 16, 17, 81, 200, 1024):
        for ties in (False, True):
            e = rng.normal(size=n)
            if ties:
                e = np.round(e * 2) / 2
                e[rng.random(n) < 0.1] = np.finfo(np.float64).max
            assert np.array_equal(H.sort_desc(e), O.sort_desc(e))


def _rand_binary(rng, h, w, p):
    img = (rng.random((h, w)) < p).astype(np.uint8)
    if rng.random() < 0.5:  # blobs with holes
        for _ in range(int(rng.integers(1, 6))):
            y0, x0 = rng.integers(0, h), rng.integers(0, w)
            y1, x1 = min(h, y0 + int(rng.integers(3, 20))), min(w, x0 + int(rng.integers(3, 20)))
            img[y0:y1, x0:x1] = 1
            img[(y0 + y1) // 2, (x0 + x1) // 2] = 0
    return img * 255


@pytest.mark.parametrize("mode", [1, 2])
def test_parallel_contours_equal_suzuki_abe(mode):
    rng = np.random.default_rng(11 + mode)
    for k in range(120):
        h, w = int(rng.integers(1, 48)), int(rng.integers(1, 48))
        img = _rand_binary(rng, h, w, rng.uniform(0.05, 0.7))
        a, ha = H.find_contours(img, mode)
        b, hb = O.find_contours(img, mode)
        assert ha == hb and len(a) == len(b)
        for u, v in zip(a, b):
            assert np.array_equal(u, v)


def test_parallel_contours_on_detector_frame():
    rng = np.random.default_rng(21)
    R, pos = synth.random_pose(rng)
    img = synth.render_host(synth.make_cam(R, pos), synth.frame_seed(9, 0))
    det = O.detector_binary(O.canny(img))
    a, ha = H.find_contours(det, 2)
    b, hb = O.find_contours(det, 2)
    assert ha == hb and len(a) == len(b) and len(a) > 50
    for u, v in zip(a, b):
        assert np.array_equal(u, v)


def test_approx_poly_dp():
    rng = np.random.default_rng(8)
    for k in range(300):
        n = int(rng.integers(1, 200))
        pts = np.cumsum(rng.integers(-3, 4, size=(n, 2)), axis=0).astype(np.int32) + 500
        for closed in (True, False):
            eps = float(rng.choice([1.0, 3.0, 10.0]))
            assert np.array_equal(H.approx_poly(pts, eps, closed), O.approx_poly(pts, eps, closed))


def test_approx_early_exit_keeps_every_quad():
    """DP output >= 10 points can never clean up to 4 (the clean-up removes at
    most every other point), so the detector stops DP there."""
    rng = np.random.default_rng(12)
    quads = 0
    contours = []
    for k in range(4):
        R, pos = synth.random_pose(rng)
        img = synth.render_host(synth.make_cam(R, pos), synth.frame_seed(9, 10 + k))
        contours += H.find_contours(O.detector_binary(O.canny(img)), 2)[0]
    for k in range(400):
        n = int(rng.integers(3, 400))
        t = np.sort(rng.uniform(0, 2 * np.pi, n))
        r = rng.uniform(20, 200) * (1 + 0.3 * np.cos(rng.integers(3, 6) * t))
        contours.append(np.column_stack([500 + r * np.cos(t), 500 + r * np.sin(t)]).astype(np.int32))
    for c in contours:
        full = O.approx_poly(c, 10.0, True)
        fast = H.approx_poly(c, 10.0, True, max_dp=10)
        if len(full) == 4:
            quads += 1
            assert fast is not None and np.array_equal(fast, full)
        else:
            assert fast is None or len(fast) != 4
    assert quads > 100


def test_bit_packed_morphology():
    rng = np.random.default_rng(31)
    for k in range(25):
        h, w = int(rng.integers(2, 90)), int(rng.integers(2, 140))
        e = (rng.random((h, w)) < rng.uniform(0.01, 0.6)).astype(np.uint8) * 255
        det, mask = H.masks_bits(e)
        assert np.array_equal(det, O.detector_binary(e) != 0)
        assert np.array_equal(mask, O.clean_mask(e) != 0)
    R, pos = synth.random_pose(rng)
    img = synth.render_host(synth.make_cam(R, pos), synth.frame_seed(9, 1))
    cn = O.canny(img)
    det, mask = H.masks_bits(cn)
    assert np.array_equal(det, O.detector_binary(cn) != 0)
    assert np.array_equal(mask, O.clean_mask(cn) != 0)


def test_fisheye_maps():
    rng = np.random.default_rng(3)
    K, D = synth.intrinsics()
    xyz = np.column_stack([rng.uniform(-3, 3, 500), rng.uniform(-3, 3, 500), rng.uniform(0.05, 3, 500)])
    assert np.array_equal(H.distort(xyz, K, D), O.distort(xyz, K, D))
    px = np.column_stack([rng.uniform(-100, 1400, 500), rng.uniform(-100, 800, 500)])
    assert np.array_equal(H.undistort(px, K, D), O.undistort(px, K, D))


def test_quad_gn_host_build_matches_restatement():
    """Per-quad GN after RPP (mk_gn.h quad_gn_refine, host build) against the
    numpy FP64 restatement (tests/_gn_ref.quad_gn_reference): same poses to
    1e-8, never a higher cost than the start, and close to the truth.
    Tolerance: 8 residuals for 6 unknowns from a 0.32 m square seen 1-2.5 m
    away leave the converged pose defined to ~1e-9 (the last accepted steps
    are at the rounding floor and their count may differ by a few between
    numpy's solve and the Cholesky; measured max 4.3e-9 over 256 problems)."""
    import _gn_ref as G
    import _hostcheck as HC

    rng = np.random.default_rng(21)
    img, obj, R0, t0, Rt, tt = G.quad_problems(rng, 64)
    R, t, steps, c0, c1 = HC.quad_gn(R0, t0, img, obj, 8)
    for i in range(len(img)):
        Rr, tr, sr, c0r, c1r = G.quad_gn_reference(R0[i], t0[i], img[i], obj[i], 8)
        np.testing.assert_allclose(R[i], Rr, atol=1e-8, rtol=0)
        np.testing.assert_allclose(t[i], tr, atol=1e-8, rtol=0)
        np.testing.assert_allclose(c0[i], c0r, rtol=1e-9)
        assert c1[i] <= c0[i]
    assert np.median(np.linalg.norm(t - tt, axis=1)) < np.median(np.linalg.norm(t0 - tt, axis=1))
    # noise-free corners: converges to the true pose
    img0, obj0, R00, t00, Rt0, tt0 = G.quad_problems(np.random.default_rng(3), 16, noise=0.0)
    R, t, steps, c0, c1 = HC.quad_gn(R00, t00, img0, obj0, 20)
    np.testing.assert_allclose(t, tt0, atol=1e-7)
    assert np.all(c1 < 1e-14)


def test_first_objpose_orientation_pairs_mirror():
    """k_objpose_q<0> runs one first ObjPose per quad: the mirrored model
    orientation's result is R diag(1, -1, -1) with identical t, errors,
    iterations and image points (host build of mk_rpp.h, bit for bit) -- on
    the quads of bench-scene frames and on random quads (the full bench set,
    38,418 quads of 128 rigs, is tools/rpp_mirror_check.py 128)."""
    import sys

    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools"))
    import rpp_mirror_check as RM
    import _gn_ref as G

    quads = RM.frame_quads(2)
    assert len(quads) > 200
    assert all(RM.mirror_pair_ok(q) for q in quads)
    img, _, _, _, _, _ = G.quad_problems(np.random.default_rng(4), 300)
    rnd = [np.vstack([p.T, np.ones(4)]) for p in img]
    assert all(RM.mirror_pair_ok(q) for q in rnd)


def test_fp32_screen_decisions_match_exact_projection():
    """The FP32 projection screen of the fast scorers (mk_screen.h, host build:
    correctly rounded reciprocals instead of the GPU's v_rcp / v_rsq, which
    tools/check_screen.hip covers on the device) never takes a decision --
    z > 0, inFrame, cvRound pixel -- that differs from the exact FP64
    projection, on the bench scene's pose distribution (truth and particle
    perturbations, every map landmark) and on arbitrary poses; and it leaves
    only a small fraction of the in-frame landmarks unsure."""
    white, red, green = synth.load_map()
    lm = np.vstack([white, red, green])
    K, D = synth.intrinsics()
    rng = np.random.default_rng(21)
    c2w, X = [], []
    for _ in range(60):
        R, pos = synth.random_pose(rng)
        for _ in range(5):
            Rp = R @ synth.rot_x(rng.normal() * 0.03) @ synth.rot_y(rng.normal() * 0.03) @ synth.rot_z(rng.normal() * 0.03)
            T = synth.truth_c2w(Rp, pos + rng.normal(size=3) * 0.01)
            c2w.append(np.repeat(T[None], len(lm), 0))
            X.append(lm)
    n_any = 100000
    Q = rng.normal(size=(n_any, 4))
    Q /= np.linalg.norm(Q, axis=1)[:, None]
    a, b, c, d = Q.T
    Rr = np.stack([a * a + b * b - c * c - d * d, 2 * (b * c - a * d), 2 * (b * d + a * c),
                   2 * (b * c + a * d), a * a - b * b + c * c - d * d, 2 * (c * d - a * b),
                   2 * (b * d - a * c), 2 * (c * d + a * b), a * a - b * b - c * c + d * d], 1).reshape(-1, 3, 3)
    Cc = rng.uniform(-3, 3, (n_any, 3))
    t = -np.einsum("nij,nj->ni", Rr, Cc)
    c2w.append(np.concatenate([Rr.reshape(-1, 9), t], 1))
    X.append(rng.uniform(-3, 3, (n_any, 3)))
    c2w = np.concatenate([np.asarray(x).reshape(-1, 12) for x in c2w])
    X = np.concatenate(X)
    bad, res = H.screen_check(c2w, X, K, D, 1280, 720)
    assert bad == 0, f"{bad} screened decisions differ from the exact projection"
    n_scene = len(X) - n_any
    inside = res[:n_scene, 1] == 1
    unsure = res[:n_scene, 0] == 2
    assert inside.sum() > 0.5 * n_scene
    assert (unsure & inside).sum() < 0.03 * inside.sum(), f"unsure {unsure.sum()} of {inside.sum()} in-frame"
    assert (res[:, 0] == 1).sum() > 0 and (res[:, 0] == 0).sum() > 0


def _sampled_screen_consts(D, n=200001):
    """Dense samples of max(theta_d', theta_d / sin theta) and of
    (1 + sum |k| theta^(2i+2)) / F over (0, pi/2] (what round 3 sampled)."""
    th = np.linspace(1.5707963267948966 / n, 1.5707963267948966, n)
    x = th * th
    k = np.asarray(D, np.float64)
    terms = np.stack([k[j] * x ** (j + 1) for j in range(4)])
    F = 1 + terms.sum(0)
    dd = 1 + sum((2 * j + 3) * terms[j] for j in range(4))
    S = max(1.0, float(np.max(np.maximum(dd, th * F / np.sin(th)))))
    M = float(np.max((1 + np.abs(terms).sum(0)) / F))
    ok = bool(np.all(dd > 0) and np.all(F > 0))
    return ok, S, M


def test_screen_bounds_derived_dominate_samples():
    """The FP32 screen's constants (mk_screen.h screen_bounds) are derived upper
    bounds: on the bench (720p), 1080p and grid1 (D = 0) intrinsics and on 10^4
    random admissible distortions, the derived S and M are >= their densely
    sampled maxima, tight (within 1 %), and the screen is disabled wherever
    the sampled curve is not increasing and positive."""
    K, D = synth.intrinsics()
    K1080 = np.array(K, np.float64).reshape(3, 3).copy()
    K1080[:2] *= 1.5
    Kg = np.array([[450, 0, 453], [0, 450, 252], [0, 0, 1]], np.float64)
    cases = [(K, D), (K1080, D), (Kg, np.zeros(4))]
    rng = np.random.default_rng(2024)
    for _ in range(10000):
        d = rng.normal(size=4) * np.array([0.05, 0.02, 0.01, 0.005]) * 10 ** rng.uniform(-2, 0.7)
        cases.append((K, d))
    n_ok = 0
    for Kc, Dc in cases:
        ok, sens, crel, S, M = H.screen_consts(Kc, Dc, 4096)
        sok, sS, sM = _sampled_screen_consts(Dc, 4097)
        if not sok:
            assert not ok  # a bound never admits a curve the samples reject
            assert np.isinf(sens)
            continue
        if not ok:
            continue  # admissible samples, but a piece's bound could not prove monotonicity: screen off (safe)
        n_ok += 1
        assert S >= sS and M >= sM, (Dc, S, sS, M, sM)
        assert S <= sS * 1.01 and M <= sM * 1.01, (Dc, S, sS, M, sM)
        f = max(float(np.asarray(Kc).reshape(9)[0]), float(np.asarray(Kc).reshape(9)[4]))
        assert abs(sens - 2.2 * S * f) <= 1e-6 * sens
        assert crel >= 24 * 2.0 ** -24 and crel >= 1.25 * (8 + 9 * M) * 2.0 ** -24 * (1 - 1e-6)
    assert n_ok > 8000, n_ok
    # the bench camera: mild distortion, M ~ 1.29, so the charge is ~24.5 u (round 3 charged 24 u)
    ok, sens, crel, S, M = H.screen_consts(K, D)
    assert ok and M < 1.5 and crel < 26 * 2.0 ** -24


def test_fp32_screen_strong_distortion_decisions():
    """The screen on strongly distorted Kannala-Brandt coefficients (theta_d
    far from theta, cancellation in 1 + k theta^2 + ...: M well above 1):
    every decision still equals the exact projection's."""
    K, _ = synth.intrinsics()
    rng = np.random.default_rng(77)
    for D in ([0.30, -0.20, 0.08, -0.012], [-0.25, 0.06, -0.004, 0.0002], [0.6, -0.5, 0.2, -0.03]):
        ok, sens, crel, S, M = H.screen_consts(K, D)
        sok, _, _ = _sampled_screen_consts(D)
        assert ok == sok
        n = 200000
        Q = rng.normal(size=(n, 4))
        Q /= np.linalg.norm(Q, axis=1)[:, None]
        a, b, c, d = Q.T
        Rr = np.stack([a * a + b * b - c * c - d * d, 2 * (b * c - a * d), 2 * (b * d + a * c),
                       2 * (b * c + a * d), a * a - b * b + c * c - d * d, 2 * (c * d - a * b),
                       2 * (b * d - a * c), 2 * (c * d + a * b), a * a - b * b - c * c + d * d], 1).reshape(-1, 3, 3)
        Cc = rng.uniform(-3, 3, (n, 3))
        t = -np.einsum("nij,nj->ni", Rr, Cc)
        c2w = np.concatenate([Rr.reshape(-1, 9), t], 1)
        X = rng.uniform(-3, 3, (n, 3))
        bad, res = H.screen_check(c2w, X, K, D, 1280, 720)
        assert bad == 0, (D, bad)
        if ok:
            assert (res[:, 0] == 1).sum() > 0  # the screen still certifies landmarks
