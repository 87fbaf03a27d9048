"""ctypes bindings for build/libmantis_hostcheck.so: the device-logic headers
(mantis_amd/csrc/mk_*.h) compiled for the host, so the per-work-item
algorithms run by the HIP kernels can be checked against the oracle on CPU.
Test infrastructure only; the product is mantis_amd/libmantis_amd.so.
"""
import ctypes as C
import os

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HC_SO = os.environ.get("MANTIS_HOSTCHECK_SO") or os.path.join(ROOT, "build", "libmantis_hostcheck.so")  # make sanitize: instrumented build
_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(HC_SO):
            raise RuntimeError("hostcheck not built: run `make tools`")
        L = C.CDLL(HC_SO)
        L.hc_rpp.restype = C.c_int
        L.hc_rpp_n.restype = C.c_int
        L.hc_rpoly.restype = C.c_int
        L.hc_approx.restype = C.c_int
        L.hc_approx.argtypes = [C.c_void_p, C.c_int, C.c_double, C.c_int, C.c_void_p, C.c_int]
        L.hc_find_contours.restype = C.c_int
        L.hc_find_contours.argtypes = [C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_void_p, C.c_int, C.c_void_p,
                                       C.c_int]
        L.hc_sort_desc.argtypes = [C.c_void_p, C.c_int, C.c_void_p]
        L.hc_distort.argtypes = [C.c_void_p, C.c_int, C.c_void_p, C.c_void_p, C.c_void_p]
        L.hc_undistort.argtypes = [C.c_void_p, C.c_int, C.c_void_p, C.c_void_p, C.c_void_p]
        L.hc_masks_bits.argtypes = [C.c_void_p, C.c_int, C.c_int, C.c_void_p, C.c_void_p]
        L.hc_gn_accumulate.argtypes = [C.c_void_p, C.c_void_p, C.c_int, C.c_void_p, C.c_int, C.c_void_p]
        L.hc_quad_gn.argtypes = [C.c_int, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_int, C.c_void_p,
                                 C.c_void_p, C.c_void_p]
        vp = C.c_void_p
        L.hc_shard_global_indices.argtypes = [C.c_int, C.c_int, vp, C.c_int, vp]
        L.hc_shard_pack_pairs.argtypes = [vp, vp, C.c_int, C.c_int, vp]
        L.hc_shard_make_recs.argtypes = [vp, vp, vp, C.c_int, C.c_int, vp]
        L.hc_shard_merge.argtypes = [vp, C.c_int, C.c_int, vp, vp]
        L.hc_rig_results.argtypes = [C.c_int, C.c_int, vp, vp, vp, vp, vp]
        L.hc_shard_offsets.restype = C.c_int64
        L.hc_shard_offsets.argtypes = [C.c_void_p, C.c_int, C.c_int, C.c_int64, C.c_void_p, C.c_void_p]
        L.hc_shard_merge.restype = C.c_int
        L.hc_screen_check.restype = C.c_int
        L.hc_screen_consts.restype = C.c_int
        L.hc_screen_consts.argtypes = [C.c_void_p, C.c_void_p, C.c_int, C.c_void_p]
        L.hc_screen_check.argtypes = [C.c_void_p, C.c_void_p, C.c_int, C.c_void_p, C.c_void_p, C.c_int, C.c_int,
                                      C.c_void_p]
        _lib = L
    return _lib


def _d(a):
    return a.ctypes.data_as(C.POINTER(C.c_double))


def rpp(model, iprts):
    model = np.ascontiguousarray(model, np.float64)
    iprts = np.ascontiguousarray(iprts, np.float64)
    assert model.shape == (3, 4) and iprts.shape == (3, 4)
    R = np.zeros(9)
    t = np.zeros(3)
    e = np.zeros(3)
    code = C.c_int(0)
    st = lib().hc_rpp(_d(model), _d(iprts), _d(R), _d(t), _d(e), C.byref(code))
    return st, R.reshape(3, 3), t, e, code.value


def rpp_n(model, iprts):
    """RPP::Rpp on 3 x n problems, n in 4..12 (the device code's host build)."""
    model = np.ascontiguousarray(model, np.float64)
    iprts = np.ascontiguousarray(iprts, np.float64)
    n = model.shape[1]
    R = np.zeros(9)
    t = np.zeros(3)
    e = np.zeros(3)
    code = C.c_int(0)
    st = lib().hc_rpp_n(_d(model), _d(iprts), C.c_int(n), _d(R), _d(t), _d(e), C.byref(code))
    return st, R.reshape(3, 3), t, e, code.value


def set_jacobi_ff(on):
    """Toggle the Jacobi noise-phase fast-forward of the host build (mk_rpp.h)."""
    lib().hc_set_jacobi_ff(C.c_int(1 if on else 0))


def rpoly(coef):
    coef = np.ascontiguousarray(coef, np.float64)
    deg = len(coef) - 1
    zr = np.zeros(deg + 1)
    zi = np.zeros(deg + 1)
    d = lib().hc_rpoly(_d(coef), C.c_int(deg), _d(zr), _d(zi))
    return d, zr, zi


def sort_desc(err):
    err = np.ascontiguousarray(err, np.float64)
    perm = np.zeros(len(err), np.int32)
    lib().hc_sort_desc(err.ctypes.data, len(err), perm.ctypes.data)
    return perm


def approx_poly(pts, eps, closed=True, max_dp=0):
    """max_dp > 0: the quad detector's early exit (returns None when it fires)."""
    pts = np.ascontiguousarray(pts, np.int32).reshape(-1, 2)
    out = np.zeros((len(pts) + 1, 2), np.int32)
    m = lib().hc_approx(pts.ctypes.data, len(pts), float(eps), int(closed), out.ctypes.data, int(max_dp))
    if m > len(pts):
        return None
    return out[:m]


def find_contours(binimg, mode):
    """mode 1 = RETR_LIST, 2 = RETR_CCOMP; returns (list of (n,2) arrays, hole flags)."""
    b = np.ascontiguousarray(binimg != 0, np.uint8)
    h, w = b.shape
    max_pts = 8 * (w + 2) * (h + 2)
    max_c = (w + 2) * (h + 2) // 2 + 8
    pts = np.zeros(2 * max_pts, np.int32)
    meta = np.zeros(3 * max_c, np.int32)
    n = lib().hc_find_contours(b.ctypes.data, w, h, mode, pts.ctypes.data, max_pts, meta.ctypes.data, max_c)
    assert n >= 0
    out, holes = [], []
    for i in range(n):
        off, cnt, hole = meta[3 * i: 3 * i + 3]
        out.append(pts[2 * off: 2 * (off + cnt)].reshape(-1, 2).copy())
        holes.append(int(hole))
    return out, holes


def distort(xyz, K, D):
    xyz = np.ascontiguousarray(xyz, np.float64).reshape(-1, 3)
    K = np.ascontiguousarray(K, np.float64).reshape(9)
    D = np.ascontiguousarray(D, np.float64).reshape(4)
    px = np.zeros((len(xyz), 2))
    lib().hc_distort(xyz.ctypes.data, len(xyz), K.ctypes.data, D.ctypes.data, px.ctypes.data)
    return px


def undistort(px, K, D):
    px = np.ascontiguousarray(px, np.float64).reshape(-1, 2)
    K = np.ascontiguousarray(K, np.float64).reshape(9)
    D = np.ascontiguousarray(D, np.float64).reshape(4)
    out = np.zeros((len(px), 2))
    lib().hc_undistort(px.ctypes.data, len(px), K.ctypes.data, D.ctypes.data, out.ctypes.data)
    return out


def masks_bits(canny_img):
    """Bit-packed detector binary (unpadded) and clean mask from a Canny image."""
    e = np.ascontiguousarray(canny_img != 0, np.uint8)
    h, w = e.shape
    det = np.zeros((h, w), np.uint8)
    mask = np.zeros((h, w), np.uint8)
    lib().hc_masks_bits(e.ctypes.data, w, h, det.ctypes.data, mask.ctypes.data)
    return det, mask


def gn_accumulate(T_w_b, T_b_c, obs):
    """mk_gn.h residual rows (the device's) summed in row order: 28 doubles."""
    T = np.ascontiguousarray(T_w_b, np.float64)
    E = np.ascontiguousarray(np.asarray(T_b_c, np.float64).reshape(-1, 16))
    o = np.ascontiguousarray(np.asarray(obs, np.float64).reshape(-1, 6))
    acc = np.zeros(28)
    lib().hc_gn_accumulate(T.ctypes.data, E.ctypes.data, len(E), o.ctypes.data, len(o), acc.ctypes.data)
    return acc


def quad_gn(R, t, img, obj, iters):
    """mk_gn.h quad_gn_refine on n problems: (R, t, steps, cost0, cost)."""
    R = np.ascontiguousarray(R, np.float64).reshape(-1, 9).copy()
    t = np.ascontiguousarray(t, np.float64).reshape(-1, 3).copy()
    img = np.ascontiguousarray(img, np.float64).reshape(-1, 8)
    obj = np.ascontiguousarray(obj, np.float64).reshape(-1, 12)
    n = len(R)
    steps = np.zeros(n, np.int32)
    c0 = np.zeros(n)
    c1 = np.zeros(n)
    lib().hc_quad_gn(n, R.ctypes.data, t.ctypes.data, img.ctypes.data, obj.ctypes.data, iters, steps.ctypes.data,
                     c0.ctypes.data, c1.ctypes.data)
    return R.reshape(n, 3, 3), t, steps, c0, c1


def screen_check(c2w, X, K, D, W, H):
    """FP32 projection screen vs the exact projection (host build of
    mk_screen.h): (mismatches, res[n, 4] = state, exact in-frame, px, py)."""
    c2w = np.ascontiguousarray(c2w, np.float64).reshape(-1, 12)
    X = np.ascontiguousarray(X, np.float64).reshape(-1, 3)
    K = np.ascontiguousarray(K, np.float64).reshape(9)
    D = np.ascontiguousarray(D, np.float64).reshape(4)
    res = np.zeros((len(X), 4), np.int32)
    bad = lib().hc_screen_check(c2w.ctypes.data, X.ctypes.data, len(X), K.ctypes.data, D.ctypes.data, W, H,
                                res.ctypes.data)
    return bad, res


def screen_consts(K, D, pieces=4096):
    """(admissible, sens, crel, S, M) of mk_screen.h screen_cam_from / screen_bounds."""
    K = np.ascontiguousarray(K, np.float64).reshape(9)
    D = np.ascontiguousarray(D, np.float64).reshape(4)
    out = np.zeros(4)
    ok = lib().hc_screen_consts(K.ctypes.data, D.ctypes.data, int(pieces), out.ctypes.data)
    return bool(ok), out[0], out[1], out[2], out[3]


# cross-rank bookkeeping of mantis_process_rig_sharded (mantis_amd/csrc/mk_shard.h)
def sizes():
    L = lib()
    return L.hc_sizeof_cam_result(), L.hc_sizeof_result(), L.hc_sizeof_shard_rec()


def shard_global_indices(n_rigs, cam_index, cams_per_rig):
    ci = np.ascontiguousarray(cam_index, np.int32)
    g = np.zeros(n_rigs * len(ci), np.int32)
    lib().hc_shard_global_indices(n_rigs, len(ci), ci.ctypes.data, cams_per_rig, g.ctypes.data)
    return g


def shard_pack_pairs(gidx, pf, slots):
    gidx = np.ascontiguousarray(gidx, np.int32)
    pf = np.ascontiguousarray(pf, np.int32)
    pairs = np.zeros(2 * slots, np.int32)
    lib().hc_shard_pack_pairs(gidx.ctypes.data, pf.ctypes.data, len(gidx), slots, pairs.ctypes.data)
    return pairs


def shard_offsets(pairs, n_global, per):
    pairs = np.ascontiguousarray(pairs, np.int32)
    flags = np.zeros(n_global, np.int32)
    off = np.zeros(n_global, np.int64)
    tot = lib().hc_shard_offsets(pairs.ctypes.data, len(pairs) // 2, n_global, per, flags.ctypes.data, off.ctypes.data)
    return flags, off, tot


def shard_make_recs(cam_bytes, tbc, gidx, slots):
    cb = np.ascontiguousarray(cam_bytes, np.uint8)
    tb = np.ascontiguousarray(tbc, np.float64).reshape(-1, 16)
    g = np.ascontiguousarray(gidx, np.int32)
    rs = sizes()[2]
    out = np.zeros(slots * rs, np.uint8)
    lib().hc_shard_make_recs(cb.ctypes.data, tb.ctypes.data, g.ctypes.data, len(g), slots, out.ctypes.data)
    return out


def shard_merge(recs, n_global):
    recs = np.ascontiguousarray(recs, np.uint8)
    cs, _, rs = sizes()
    allb = np.zeros(n_global * cs, np.uint8)
    tall = np.zeros((n_global, 16))
    code = lib().hc_shard_merge(recs.ctypes.data, len(recs) // rs, n_global, allb.ctypes.data, tall.ctypes.data)
    return code, allb.reshape(n_global, cs), tall


def rig_results(n_rigs, cams_per_rig, all_bytes, tall, pf, states):
    ab = np.ascontiguousarray(all_bytes, np.uint8)
    tb = np.ascontiguousarray(tall, np.float64)
    pf = np.ascontiguousarray(pf, np.int32)
    st = np.ascontiguousarray(states, np.uint64)
    out = np.zeros(n_rigs * sizes()[1], np.uint8)
    lib().hc_rig_results(n_rigs, cams_per_rig, ab.ctypes.data, tb.ctypes.data, pf.ctypes.data, st.ctypes.data,
                         out.ctypes.data)
    return out.reshape(n_rigs, -1)
