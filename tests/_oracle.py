"""ctypes bindings for the ORACLE (test infrastructure only).

Loads oracle/liboracle.so (CPU restatement of the reference mantis3 path) and,
when present, oracle/_ref/libref_rpoly.so (the reference's own Rpoly.cpp
compiled in place; RPP.cpp needs OpenCV and is not built).  Only tests/, __graft_entry__.smoke()
and bench.py's cpu_baseline use this module.
"""
import ctypes as C
import os

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_SO = os.environ.get("MANTIS_ORACLE_SO") or os.path.join(ROOT, "oracle", "liboracle.so")  # make sanitize: instrumented build
REF_SO = os.path.join(ROOT, "oracle", "_ref", "libref_rpoly.so")

ORC_MAX_QUADS = 256
ORC_MAX_HYPS = 1024


class OrcFrameDebug(C.Structure):
    _fields_ = [
        ("reason", C.c_int32), ("publish", C.c_int32), ("n_raw_quads", C.c_int32), ("n_quads", C.c_int32),
        ("quads", (C.c_int32 * 8) * ORC_MAX_QUADS), ("test_pts", (C.c_double * 8) * ORC_MAX_QUADS),
        ("n_gen", C.c_int32), ("n_hyps", C.c_int32),
        ("hyp_c2w", (C.c_double * 12) * ORC_MAX_HYPS), ("hyp_err", C.c_double * ORC_MAX_HYPS),
        ("hyp_n", C.c_int32 * ORC_MAX_HYPS),
        ("best1_c2w", C.c_double * 12), ("best1_err", C.c_double),
        ("pf_c2w", C.c_double * 12), ("pf_err", C.c_double), ("pf_iter_err", C.c_double * 11),
        ("shift_err", C.c_double * 81), ("top20_err", C.c_double * 20), ("yaw_err", C.c_double * 4),
        ("yaw_best", C.c_int32), ("min_yaw_diff", C.c_double), ("pub_c2w", C.c_double * 12),
        ("pub_error", C.c_double), ("position", C.c_double * 3), ("orientation_xyzw", C.c_double * 4),
        ("covariance", C.c_double * 36), ("rng_state_after", C.c_uint64), ("n_scored", C.c_int32),
    ]


def _p(a, t):
    return a.ctypes.data_as(C.POINTER(t))


_lib = None
_ref = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(ORACLE_SO):
            raise RuntimeError("oracle not built: run `make -C oracle` (or __graft_entry__.build())")
        L = C.CDLL(ORACLE_SO)
        L.orc_create.restype = C.c_void_p
        L.orc_create.argtypes = [C.c_void_p, C.c_int32, C.c_void_p, C.c_int32, C.c_void_p, C.c_int32, C.c_uint64]
        L.orc_destroy.argtypes = [C.c_void_p]
        L.orc_rng_get.restype = C.c_uint64
        L.orc_rng_get.argtypes = [C.c_void_p]
        L.orc_rng_set.argtypes = [C.c_void_p, C.c_uint64]
        L.orc_process_frame.argtypes = [C.c_void_p, C.c_void_p, C.c_int32, C.c_int32, C.c_int32, C.c_void_p,
                                        C.c_void_p, C.POINTER(OrcFrameDebug)]
        L.orc_find_contours.restype = C.c_int32
        L.orc_approx_poly.restype = C.c_int32
        L.orc_parse_coordinates.restype = C.c_int32
        L.orc_parse_coordinates.argtypes = [C.c_char_p, C.c_void_p, C.c_int32]
        L.orc_rpp.restype = C.c_int32
        L.orc_rpoly.restype = C.c_int32
        L.orc_gaussians.restype = C.c_uint64
        L.orc_gaussians.argtypes = [C.c_uint64, C.c_int32, C.c_void_p]
        L.orc_approx_poly.argtypes = [C.c_void_p, C.c_int32, C.c_double, C.c_int32, C.c_void_p]
        L.orc_camera_error.argtypes = [C.c_void_p, C.c_void_p, C.c_int32, C.c_int32, C.c_void_p, C.c_void_p,
                                       C.c_void_p, C.c_int32, C.c_void_p, C.c_void_p]
        L.orc_markov_init.argtypes = [C.c_void_p, C.c_void_p]
        L.orc_markov_sense.argtypes = [C.c_void_p, C.c_void_p]
        L.orc_markov_convolve.argtypes = [C.c_void_p, C.c_double, C.c_double]
        L.orc_markov_weight.argtypes = [C.c_void_p, C.c_void_p, C.c_int32, C.c_void_p]
        L.orc_markov_yaw.argtypes = [C.c_void_p, C.c_void_p]
        L.orc_markov_yaw.restype = C.c_double
        L.orc_markov_bin.argtypes = [C.c_void_p]
        L.orc_markov_bin.restype = C.c_int32
        L.orc_score.argtypes = [C.c_void_p, C.c_void_p, C.c_int32, C.c_int32, C.c_void_p, C.c_void_p, C.c_void_p,
                                C.c_int32, C.c_int32, C.c_void_p, C.c_void_p]
        _lib = L
    return _lib


def ref():
    """The reference's own Rpoly (None when oracle/_ref was not built)."""
    global _ref
    if _ref is None and os.path.exists(REF_SO):
        R = C.CDLL(REF_SO)
        R.ref_rpoly.restype = C.c_int
        _ref = R
    return _ref


# ------------------------------------------------------------------ helpers
def rpp(model, iprts):
    model = np.ascontiguousarray(model, np.float64)
    iprts = np.ascontiguousarray(iprts, np.float64)
    n = model.shape[1]
    R = np.zeros(9)
    t = np.zeros(3)
    e = np.zeros(3)
    code = C.c_int32(0)
    st = lib().orc_rpp(_p(model, C.c_double), _p(iprts, C.c_double), n, _p(R, C.c_double), _p(t, C.c_double),
                       _p(e, C.c_double), C.byref(code))
    return st, R.reshape(3, 3), t, e, code.value


def rpoly(coef, ref_impl=False):
    coef = np.ascontiguousarray(coef, np.float64)
    deg = len(coef) - 1
    zr = np.zeros(deg + 1)
    zi = np.zeros(deg + 1)
    if ref_impl:
        d = ref().ref_rpoly(_p(coef, C.c_double), C.c_int(deg), _p(zr, C.c_double), _p(zi, C.c_double))
    else:
        d = lib().orc_rpoly(_p(coef, C.c_double), C.c_int32(deg), _p(zr, C.c_double), _p(zi, C.c_double))
    return d, zr, zi


def gaussians(state, n):
    out = np.zeros(n, np.float32)
    st = lib().orc_gaussians(C.c_uint64(state), n, _p(out, C.c_float))
    return out, st


def parse_coordinates(s):
    buf = np.zeros(3 * 4096)
    n = lib().orc_parse_coordinates(s.encode(), _p(buf, C.c_double), 4096)
    return buf[: 3 * n].reshape(n, 3)


def canny(bgr):
    h, w = bgr.shape[:2]
    out = np.zeros((h, w), np.uint8)
    bgr = np.ascontiguousarray(bgr)
    lib().orc_canny(_p(bgr, C.c_uint8), C.c_int32(w), C.c_int32(h), C.c_int32(3 * w), _p(out, C.c_uint8))
    return out


def hysteresis(cls):
    """cv::Canny's hysteresis walk on a class plane (0 none, 1 weak candidate, 2 strong)."""
    cls = np.ascontiguousarray(cls, np.uint8)
    h, w = cls.shape
    out = np.zeros((h, w), np.uint8)
    lib().orc_hysteresis(_p(cls, C.c_uint8), C.c_int32(w), C.c_int32(h), _p(out, C.c_uint8))
    return out


def gray(bgr):
    h, w = bgr.shape[:2]
    out = np.zeros((h, w), np.uint8)
    bgr = np.ascontiguousarray(bgr)
    lib().orc_gray(_p(bgr, C.c_uint8), C.c_int32(w), C.c_int32(h), C.c_int32(3 * w), _p(out, C.c_uint8))
    return out


def blur(g):
    h, w = g.shape
    out = np.zeros((h, w), np.uint8)
    g = np.ascontiguousarray(g)
    lib().orc_blur(_p(g, C.c_uint8), C.c_int32(w), C.c_int32(h), _p(out, C.c_uint8))
    return out


def detector_binary(canny_img):
    h, w = canny_img.shape
    out = np.zeros((h, w), np.uint8)
    c = np.ascontiguousarray(canny_img)
    lib().orc_detector_binary(_p(c, C.c_uint8), C.c_int32(w), C.c_int32(h), _p(out, C.c_uint8))
    return out


def clean_mask(canny_img):
    h, w = canny_img.shape
    out = np.zeros((h, w), np.uint8)
    c = np.ascontiguousarray(canny_img)
    lib().orc_clean_mask(_p(c, C.c_uint8), C.c_int32(w), C.c_int32(h), _p(out, C.c_uint8))
    return out


def find_contours(binimg, mode):
    h, w = binimg.shape
    b = np.ascontiguousarray(binimg, np.uint8)
    max_pts, max_c = 4 * w * h + 16, w * h // 2 + 16
    pts = np.zeros(2 * max_pts, np.int32)
    meta = np.zeros(3 * max_c, np.int32)
    n = lib().orc_find_contours(_p(b, C.c_uint8), C.c_int32(w), C.c_int32(h), C.c_int32(mode), _p(pts, C.c_int32),
                                C.c_int32(max_pts), _p(meta, C.c_int32), C.c_int32(max_c))
    assert n >= 0
    out, holes = [], []
    for i in range(n):
        o, c, hole = meta[3 * i: 3 * i + 3]
        out.append(pts[2 * o: 2 * (o + c)].reshape(c, 2).copy())
        holes.append(int(hole))
    return out, holes


def approx_poly(pts, eps, closed=True):
    pts = np.ascontiguousarray(pts, np.int32)
    out = np.zeros_like(pts)
    n = lib().orc_approx_poly(_p(pts, C.c_int32), len(pts), eps, int(closed), _p(out, C.c_int32))
    return out[:n].copy()


def sort_desc(err):
    err = np.ascontiguousarray(err, np.float64)
    perm = np.zeros(len(err), np.int32)
    lib().orc_sort_desc(_p(err, C.c_double), C.c_int32(len(err)), _p(perm, C.c_int32))
    return perm


def distort(xyz, K, D):
    xyz = np.ascontiguousarray(xyz, np.float64).reshape(-1, 3)
    K = np.ascontiguousarray(K, np.float64).reshape(9)
    D = np.ascontiguousarray(D, np.float64).reshape(4)
    px = np.zeros((len(xyz), 2))
    lib().orc_distort(_p(xyz, C.c_double), C.c_int32(len(xyz)), _p(K, C.c_double), _p(D, C.c_double),
                      _p(px, C.c_double))
    return px


def undistort(px, K, D):
    px = np.ascontiguousarray(px, np.float64).reshape(-1, 2)
    K = np.ascontiguousarray(K, np.float64).reshape(9)
    D = np.ascontiguousarray(D, np.float64).reshape(4)
    out = np.zeros((len(px), 2))
    lib().orc_undistort(_p(px, C.c_double), C.c_int32(len(px)), _p(K, C.c_double), _p(D, C.c_double),
                        _p(out, C.c_double))
    return out


class Markov:
    """Oracle restatement of MarkovModel (oracle/o_markov.cpp), one plane."""

    def __init__(self, w2c_R):
        self.p = np.zeros(360)
        R = np.ascontiguousarray(w2c_R, np.float64).reshape(9)
        lib().orc_markov_init(R.ctypes.data, self.p.ctypes.data)

    def sense(self, w2c_R):
        R = np.ascontiguousarray(w2c_R, np.float64).reshape(9)
        lib().orc_markov_sense(self.p.ctypes.data, R.ctypes.data)

    def convolve(self, dtheta, dt):
        lib().orc_markov_convolve(self.p.ctypes.data, C.c_double(dtheta), C.c_double(dt))

    def weight(self, w2c_R, error):
        R = np.ascontiguousarray(w2c_R, np.float64).reshape(-1, 9)
        e = np.ascontiguousarray(error, np.float64).copy()
        lib().orc_markov_weight(self.p.ctypes.data, R.ctypes.data, len(R), e.ctypes.data)
        return e

    def yaw(self):
        am = C.c_int32()
        y = lib().orc_markov_yaw(self.p.ctypes.data, C.byref(am))
        return y, am.value

    @staticmethod
    def bin(w2c_R):
        R = np.ascontiguousarray(w2c_R, np.float64).reshape(9)
        return lib().orc_markov_bin(R.ctypes.data)


class Oracle:
    """One oracle context: map + the global cv::RNG(1) of Mantis3Params.h:87."""

    def __init__(self, white, red, green, seed=1):
        L = lib()
        self._w = np.ascontiguousarray(white, np.float64)
        self._r = np.ascontiguousarray(red, np.float64)
        self._g = np.ascontiguousarray(green, np.float64)
        self.ctx = L.orc_create(self._w.ctypes.data, len(self._w), self._r.ctypes.data, len(self._r),
                                self._g.ctypes.data, len(self._g), C.c_uint64(seed))

    def __del__(self):
        try:
            lib().orc_destroy(self.ctx)
        except Exception:
            pass

    @property
    def rng_state(self):
        return lib().orc_rng_get(self.ctx)

    @rng_state.setter
    def rng_state(self, s):
        lib().orc_rng_set(self.ctx, C.c_uint64(s))

    def process(self, bgr, K, D):
        h, w = bgr.shape[:2]
        bgr = np.ascontiguousarray(bgr, np.uint8)
        K = np.ascontiguousarray(K, np.float64).reshape(9)
        D = np.ascontiguousarray(D, np.float64).reshape(4)
        dbg = OrcFrameDebug()
        lib().orc_process_frame(self.ctx, bgr.ctypes.data, w, h, 3 * w, K.ctypes.data, D.ctypes.data, C.byref(dbg))
        return dbg

    def camera_error(self, bgr, K, D, c2w, colors=(255, 255, 255, 50, 85, 255, 50, 255, 85)):
        """Legacy MonteCarlo::computeCameraError raw sums: (error sum, count) per pose."""
        h, w = bgr.shape[:2]
        bgr = np.ascontiguousarray(bgr, np.uint8)
        K = np.ascontiguousarray(K, np.float64).reshape(9)
        D = np.ascontiguousarray(D, np.float64).reshape(4)
        c2w = np.ascontiguousarray(c2w, np.float64).reshape(-1, 12)
        col = np.ascontiguousarray(colors, np.int32)
        sums = np.zeros((len(c2w), 2))
        lib().orc_camera_error(self.ctx, bgr.ctypes.data, w, h, K.ctypes.data, D.ctypes.data, c2w.ctypes.data,
                               len(c2w), col.ctypes.data, sums.ctypes.data)
        return sums

    def score(self, bgr, K, D, c2w, fast=True):
        h, w = bgr.shape[:2]
        bgr = np.ascontiguousarray(bgr, np.uint8)
        K = np.ascontiguousarray(K, np.float64).reshape(9)
        D = np.ascontiguousarray(D, np.float64).reshape(4)
        c2w = np.ascontiguousarray(c2w, np.float64).reshape(-1, 12)
        n = len(c2w)
        err = np.zeros(n)
        npj = np.zeros(n, np.int32)
        lib().orc_score(self.ctx, bgr.ctypes.data, w, h, K.ctypes.data, D.ctypes.data, c2w.ctypes.data, n,
                        int(fast), err.ctypes.data, npj.ctypes.data)
        return err, npj
