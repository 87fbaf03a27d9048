"""mantis_amd — MI355X-native mantis3 hot path.

Python is only a thin ctypes view of the C-ABI in include/mantis.h, used by
tests/, bench.py and __graft_entry__.py; the product is libmantis_amd.so
(HIP kernels for gfx950 + C++ host orchestration). There is no CPU fallback:
loading fails loudly when the library is missing, and mantis_create fails
when no GPU is present.
"""
import ctypes as C
import os

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB_PATH = os.environ.get("MANTIS_AMD_LIB") or os.path.join(os.path.dirname(os.path.abspath(__file__)),
                                                             "libmantis_amd.so")

MANTIS_OK = 0
REASONS = {0: "published", 1: "no_quads", 2: "no_hyps", 3: "yaw_ambiguous", 4: "no_yaw"}


class MantisConfig(C.Structure):
    _fields_ = [("struct_size", C.c_int32), ("device", C.c_int32), ("max_cams", C.c_int32),
                ("max_width", C.c_int32), ("max_height", C.c_int32), ("rng_seed", C.c_uint64),
                ("canny_low", C.c_int32), ("polygon_epsilon", C.c_int32),
                ("search_radius_multiplier", C.c_double), ("grid_spacing", C.c_double),
                ("particles", C.c_int32), ("iterations", C.c_int32), ("gn_enable", C.c_int32),
                ("gn_iterations", C.c_int32), ("max_quads", C.c_int32), ("max_contour_points", C.c_int32),
                ("quad_gn_iterations", C.c_int32), ("rig_weighting", C.c_int32)]


class MantisImage(C.Structure):
    _fields_ = [("width", C.c_int32), ("height", C.c_int32), ("step_bytes", C.c_int32), ("mem_kind", C.c_int32),
                ("bgr", C.c_void_p), ("K", C.c_double * 9), ("D", C.c_double * 4),
                ("T_base_cam", C.c_double * 16), ("stamp_ns", C.c_int64), ("frame_id", C.c_char_p)]


class MantisMotion(C.Structure):
    _fields_ = [("delta_pos", C.c_double * 3), ("delta_quat_xyzw", C.c_double * 4)]


class MantisCamResult(C.Structure):
    _fields_ = [("status", C.c_int32), ("reason", C.c_int32), ("publish", C.c_int32), ("n_quads", C.c_int32),
                ("n_hyps", C.c_int32), ("n_scored", C.c_int32), ("position", C.c_double * 3),
                ("orientation_xyzw", C.c_double * 4), ("covariance", C.c_double * 36), ("error", C.c_double),
                ("min_yaw_diff", C.c_double), ("pf_error", C.c_double), ("c2w", C.c_double * 12)]


class MantisResult(C.Structure):
    _fields_ = [("status", C.c_int32), ("publish", C.c_int32), ("n_cams_published", C.c_int32),
                ("num_particles", C.c_int32), ("position", C.c_double * 3), ("orientation_xyzw", C.c_double * 4),
                ("covariance", C.c_double * 36), ("weight", C.c_double), ("min_yaw_diff", C.c_double),
                ("n_quads", C.c_int32), ("gn_iterations", C.c_int32), ("gn_cost", C.c_double),
                ("rng_state_after", C.c_uint64)]


class MantisRigGnInfo(C.Structure):
    _fields_ = [("T_init", C.c_double * 16), ("T_final", C.c_double * 16), ("cost0", C.c_double),
                ("cost", C.c_double), ("valid", C.c_int32), ("iterations", C.c_int32), ("n_obs", C.c_int32),
                ("n_obs_local", C.c_int32)]


class SynthCamC(C.Structure):
    _fields_ = [("fx", C.c_double), ("fy", C.c_double), ("cx", C.c_double), ("cy", C.c_double),
                ("k", C.c_double * 4), ("R_wc", C.c_double * 9), ("pos", C.c_double * 3),
                ("w", C.c_int32), ("h", C.c_int32), ("pad", C.c_int32 * 2)]


class FrameDebug(C.Structure):
    """Layout of mk::FrameDebug == oracle orc_frame_debug."""
    _fields_ = [
        ("reason", C.c_int32), ("publish", C.c_int32), ("n_raw_quads", C.c_int32), ("n_quads", C.c_int32),
        ("quads", (C.c_int32 * 8) * 256), ("test_pts", (C.c_double * 8) * 256),
        ("n_gen", C.c_int32), ("n_hyps", C.c_int32),
        ("hyp_c2w", (C.c_double * 12) * 1024), ("hyp_err", C.c_double * 1024), ("hyp_n", C.c_int32 * 1024),
        ("best1_c2w", C.c_double * 12), ("best1_err", C.c_double),
        ("pf_c2w", C.c_double * 12), ("pf_err", C.c_double), ("pf_iter_err", C.c_double * 11),
        ("shift_err", C.c_double * 81), ("top20_err", C.c_double * 20), ("yaw_err", C.c_double * 4),
        ("yaw_best", C.c_int32), ("min_yaw_diff", C.c_double), ("pub_c2w", C.c_double * 12),
        ("pub_error", C.c_double), ("position", C.c_double * 3), ("orientation_xyzw", C.c_double * 4),
        ("covariance", C.c_double * 36), ("rng_state_after", C.c_uint64), ("n_scored", C.c_int32),
    ]


_lib = None

_SIGS = {
    "mantis_abi_version": (C.c_int32, []),
    "mantis_default_config": (None, [C.POINTER(MantisConfig)]),
    "mantis_create": (C.c_int, [C.POINTER(MantisConfig), C.POINTER(C.c_void_p)]),
    "mantis_destroy": (C.c_int, [C.c_void_p]),
    "mantis_last_error": (C.c_char_p, [C.c_void_p]),
    "mantis_set_map": (C.c_int, [C.c_void_p, C.c_void_p, C.c_int32, C.c_void_p, C.c_int32, C.c_void_p, C.c_int32]),
    "mantis_parse_coordinates": (C.c_int32, [C.c_char_p, C.c_void_p, C.c_int32]),
    "mantis_rng_get": (C.c_int, [C.c_void_p, C.POINTER(C.c_uint64)]),
    "mantis_rng_set": (C.c_int, [C.c_void_p, C.c_uint64]),
    "mantis_process": (C.c_int, [C.c_void_p, C.POINTER(MantisImage), C.c_int32, C.POINTER(MantisMotion),
                                 C.POINTER(MantisResult), C.POINTER(MantisCamResult)]),
    "mantis_process_batch": (C.c_int, [C.c_void_p, C.POINTER(MantisImage), C.c_int32, C.c_int32,
                                       C.POINTER(MantisResult), C.POINTER(MantisCamResult)]),
    "mantis_canny": (C.c_int, [C.c_void_p, C.POINTER(MantisImage), C.c_void_p]),
    "mantis_hysteresis": (C.c_int, [C.c_void_p, C.c_void_p, C.c_int32, C.c_int32, C.c_void_p]),
    "mantis_masks": (C.c_int, [C.c_void_p, C.POINTER(MantisImage), C.c_void_p, C.c_void_p]),
    "mantis_detect_quads": (C.c_int, [C.c_void_p, C.POINTER(MantisImage), C.c_void_p, C.c_int32,
                                      C.POINTER(C.c_int32)]),
    "mantis_score_hypotheses": (C.c_int, [C.c_void_p, C.POINTER(MantisImage), C.c_void_p, C.c_void_p, C.c_int32,
                                          C.c_int32, C.c_void_p, C.c_void_p]),
    "mantis_rpp_batch": (C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_int32, C.c_void_p, C.c_void_p,
                                   C.c_void_p, C.c_void_p]),
    "mantis_small_batch_frames": (C.c_int32, [C.c_void_p]),
    "mantis_rpp_solve": (C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_int32, C.c_int32, C.c_void_p,
                                   C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p]),
    "mantis_quad_gn": (C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_int32, C.c_void_p, C.c_void_p, C.c_int32,
                                 C.c_void_p, C.c_void_p]),
    "mantis_get_rig_weights": (C.c_int, [C.c_void_p, C.c_int32, C.c_void_p, C.c_void_p, C.c_void_p,
                                         C.POINTER(C.c_int32)]),
    "mantis_markov_init": (C.c_int, [C.c_void_p, C.c_int32, C.c_void_p]),
    "mantis_markov_sense": (C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p]),
    "mantis_markov_convolve": (C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p]),
    "mantis_markov_weight": (C.c_int, [C.c_void_p, C.c_int32, C.c_void_p, C.c_int32, C.c_void_p]),
    "mantis_markov_get": (C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p]),
    "mantis_set_prior_pose": (C.c_int, [C.c_void_p, C.c_void_p]),
    "mantis_get_prior_pose": (C.c_int, [C.c_void_p, C.c_void_p, C.POINTER(C.c_int32)]),
    "mantis_synth_render": (C.c_int, [C.c_void_p, C.POINTER(SynthCamC), C.c_int32, C.c_void_p, C.c_void_p]),
    "mantis_device_alloc": (C.c_int, [C.c_void_p, C.c_size_t, C.POINTER(C.c_void_p)]),
    "mantis_device_free": (C.c_int, [C.c_void_p, C.c_void_p]),
    "mantis_memcpy_h2d": (C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_size_t]),
    "mantis_memcpy_d2h": (C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_size_t]),
    "mantis_synchronize": (C.c_int, [C.c_void_p]),
    "mantis_kernel_times": (C.c_int32, [C.c_void_p, C.POINTER(C.c_char_p), C.POINTER(C.c_float), C.c_int32]),
    "mantis_set_profiling": (C.c_int, [C.c_void_p, C.c_int32]),
    "mantis_frame_debug_size": (C.c_size_t, []),
    "mantis_get_frame_debug": (C.c_int, [C.c_void_p, C.c_int32, C.c_void_p, C.c_size_t]),
    "mantis_get_contours": (C.c_int, [C.c_void_p, C.c_int32, C.c_void_p, C.c_void_p, C.c_int32, C.c_void_p, C.c_int32,
                                      C.c_void_p]),
    "mantis_frame_counters": (C.c_int32, [C.c_void_p, C.c_int32, C.c_void_p, C.c_int32]),
    "mantis_gn_accumulate": (C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_int32, C.c_void_p, C.c_int32,
                                       C.c_void_p]),
    "mantis_gn_solve": (C.c_int, [C.c_void_p, C.c_double, C.c_void_p, C.c_void_p]),
    "mantis_comm_unique_id": (C.c_int, [C.c_void_p]),
    "mantis_comm_init": (C.c_int, [C.c_void_p, C.c_void_p, C.c_int32, C.c_int32]),
    "mantis_comm_info": (C.c_int, [C.c_void_p, C.POINTER(C.c_int32), C.POINTER(C.c_int32)]),
    "mantis_process_rig_sharded": (C.c_int, [C.c_void_p, C.POINTER(MantisImage), C.c_int32, C.c_int32, C.c_void_p,
                                             C.c_int32, C.POINTER(MantisResult), C.POINTER(MantisCamResult)]),
    "mantis_get_rig_gn": (C.c_int, [C.c_void_p, C.c_int32, C.POINTER(MantisRigGnInfo), C.c_void_p, C.c_int32]),
    "mantis_gn_allreduce": (C.c_int, [C.c_void_p, C.c_void_p]),
    "mantis_score_argmin": (C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_int32, C.c_int64,
                                      C.c_int32, C.c_void_p, C.c_void_p]),
    "mantis_score_argmin_dev": (C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_int32, C.c_int64,
                                      C.c_int32, C.c_void_p, C.c_void_p]),
    "mantis_argmin_pick": (C.c_int, [C.c_void_p, C.c_int32, C.c_void_p, C.c_void_p]),
    "mantis_score_argmin_batch": (C.c_int, [C.c_void_p, C.c_void_p, C.c_int32, C.c_void_p, C.c_void_p, C.c_void_p,
                                            C.c_void_p, C.c_int32, C.c_void_p, C.c_void_p]),
    "mantis_get_rig_weights_info": (C.c_int, [C.c_void_p, C.POINTER(C.c_int32), C.POINTER(C.c_int32)]),
    "mantis_shard_gauss_offsets": (C.c_int, [C.c_void_p, C.c_void_p, C.c_int32, C.c_int32, C.c_void_p, C.c_int32,
                                             C.c_int32, C.c_void_p, C.POINTER(C.c_int32)]),
}


# include/mantis_ros.h (ROS side of the drop-in; mirrored in mantis_amd/ros.py)
class RosHeader(C.Structure):
    _fields_ = [("seq", C.c_uint32), ("stamp_sec", C.c_uint32), ("stamp_nsec", C.c_uint32),
                ("frame_id", C.c_void_p), ("frame_id_len", C.c_uint32)]


class RosImage(C.Structure):
    _fields_ = [("header", RosHeader), ("height", C.c_uint32), ("width", C.c_uint32), ("encoding", C.c_void_p),
                ("encoding_len", C.c_uint32), ("is_bigendian", C.c_uint8), ("step", C.c_uint32),
                ("data", C.c_void_p), ("data_len", C.c_uint32)]


class RosCameraInfo(C.Structure):
    _fields_ = [("header", RosHeader), ("height", C.c_uint32), ("width", C.c_uint32),
                ("distortion_model", C.c_void_p), ("distortion_model_len", C.c_uint32), ("D_len", C.c_uint32),
                ("D", C.c_double * 16), ("K", C.c_double * 9), ("R", C.c_double * 9), ("P", C.c_double * 12),
                ("binning_x", C.c_uint32), ("binning_y", C.c_uint32), ("roi_x_offset", C.c_uint32),
                ("roi_y_offset", C.c_uint32), ("roi_height", C.c_uint32), ("roi_width", C.c_uint32),
                ("roi_do_rectify", C.c_uint8)]


class RosPoseStamped(C.Structure):
    _fields_ = [("seq", C.c_uint32), ("stamp_sec", C.c_uint32), ("stamp_nsec", C.c_uint32),
                ("frame_id", C.c_char * 32), ("position", C.c_double * 3), ("orientation_xyzw", C.c_double * 4),
                ("covariance", C.c_double * 36)]


class RosServiceResponse(C.Structure):
    _fields_ = [("position", C.c_double * 3), ("orientation_xyzw", C.c_double * 4), ("weight", C.c_double),
                ("num_particles", C.c_int32)]


_SIGS.update({
    "mantis_ros_parse_image": (C.c_int64, [C.c_void_p, C.c_size_t, C.POINTER(RosImage)]),
    "mantis_ros_parse_camera_info": (C.c_int64, [C.c_void_p, C.c_size_t, C.POINTER(RosCameraInfo)]),
    "mantis_ros_parse_service_request": (C.c_int64, [C.c_void_p, C.c_size_t, C.POINTER(RosImage),
                                                     C.POINTER(C.c_int32), C.POINTER(RosCameraInfo),
                                                     C.POINTER(C.c_int32), C.c_int32, C.POINTER(MantisMotion)]),
    "mantis_ros_write_pose": (C.c_int64, [C.POINTER(RosPoseStamped), C.c_void_p, C.c_size_t]),
    "mantis_ros_write_service_response": (C.c_int64, [C.POINTER(RosServiceResponse), C.c_void_p, C.c_size_t]),
    "mantis_ros_to_image": (C.c_int, [C.POINTER(RosImage), C.POINTER(RosCameraInfo), C.POINTER(MantisImage)]),
    "mantis_ros_pose_from_result": (C.c_int32, [C.POINTER(MantisCamResult), C.POINTER(RosHeader), C.c_int32,
                                                C.POINTER(RosPoseStamped)]),
    "mantis_ros_service_response_from_result": (C.c_int, [C.POINTER(MantisResult),
                                                           C.POINTER(RosServiceResponse)]),
    "mantis_ros_image_callback": (C.c_int, [C.c_void_p, C.c_void_p, C.c_size_t, C.c_void_p, C.c_size_t, C.c_int32,
                                            C.c_void_p, C.c_size_t, C.POINTER(C.c_int64),
                                            C.POINTER(MantisCamResult)]),
    "mantis_ros_service_call": (C.c_int, [C.c_void_p, C.c_void_p, C.c_size_t, C.c_void_p, C.c_size_t,
                                          C.POINTER(C.c_int64), C.POINTER(MantisResult)]),
})


def lib():
    """Load libmantis_amd.so (raises if it was not built)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(f"{LIB_PATH} missing: build it with __graft_entry__.build() (hipcc, gfx950)")
        L = C.CDLL(LIB_PATH)
        for name, (res, args) in _SIGS.items():
            if not hasattr(L, name) and os.environ.get("MANTIS_AMD_LIB"):
                continue  # an older library under A/B (MANTIS_AMD_LIB): entry points it lacks stay unbound
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        _lib = L
    return _lib


class MantisError(RuntimeError):
    pass


def default_config(**kw):
    cfg = MantisConfig()
    lib().mantis_default_config(C.byref(cfg))
    for k, v in kw.items():
        setattr(cfg, k, v)
    return cfg


def make_image(bgr, K, D, T_base_cam=None, device_ptr=None, width=None, height=None):
    """mantis_image for a host numpy BGR8 array or a device pointer."""
    im = MantisImage()
    if device_ptr is not None:
        im.width, im.height = width, height
        im.step_bytes = 3 * width
        im.mem_kind = 1
        im.bgr = device_ptr
    else:
        assert bgr.dtype == np.uint8 and bgr.ndim == 3 and bgr.shape[2] == 3
        bgr = np.ascontiguousarray(bgr)
        im.height, im.width = bgr.shape[:2]
        im.step_bytes = bgr.strides[0]
        im.mem_kind = 0
        im.bgr = bgr.ctypes.data
        im._keep = bgr
    Kf = np.asarray(K, np.float64).reshape(9)
    for i in range(9):
        im.K[i] = Kf[i]
    Df = np.asarray(D, np.float64).reshape(4)
    for i in range(4):
        im.D[i] = Df[i]
    T = np.eye(4) if T_base_cam is None else np.asarray(T_base_cam, np.float64)
    for i in range(16):
        im.T_base_cam[i] = T.reshape(16)[i]
    return im


class Batch:
    """mantis_process_batch arguments built once (the bench's throughput path:
    no per-call Python conversion of thousands of ctypes records). run() is
    one C call (ctypes releases the GIL); results stay in .out / .cam_out."""

    def __init__(self, ctx, images, rigs):
        self.ctx, self.n, self.rigs = ctx, len(images), rigs
        self.cams = (MantisImage * self.n)(*images)
        self.out = (MantisResult * rigs)()
        self.cam_out = (MantisCamResult * self.n)()

    def run(self):
        st = lib().mantis_process_batch(self.ctx.h, self.cams, self.rigs, self.n // self.rigs, self.out, self.cam_out)
        self.ctx._chk(st, "process_batch")


class Mantis:
    """One mantis_amd context (one GPU, one HIP stream, one cv::RNG stream)."""

    def __init__(self, cfg=None, **kw):
        L = lib()
        self.cfg = cfg if cfg is not None else default_config(**kw)
        h = C.c_void_p()
        st = L.mantis_create(C.byref(self.cfg), C.byref(h))
        if st != MANTIS_OK:
            raise MantisError(f"mantis_create failed ({st}): {L.mantis_last_error(None).decode()}")
        self.h = h

    def close(self):
        if getattr(self, "h", None):
            lib().mantis_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _chk(self, st, what):
        if st != MANTIS_OK:
            raise MantisError(f"{what} failed ({st}): {lib().mantis_last_error(self.h).decode()}")

    def set_map(self, white, red, green):
        self._map = [np.ascontiguousarray(a, np.float64) for a in (white, red, green)]
        w, r, g = self._map
        self._chk(lib().mantis_set_map(self.h, w.ctypes.data, len(w), r.ctypes.data, len(r), g.ctypes.data, len(g)),
                  "set_map")

    @property
    def rng_state(self):
        v = C.c_uint64()
        self._chk(lib().mantis_rng_get(self.h, C.byref(v)), "rng_get")
        return v.value

    @rng_state.setter
    def rng_state(self, s):
        self._chk(lib().mantis_rng_set(self.h, C.c_uint64(s)), "rng_set")

    def process(self, images, rigs=1):
        n = len(images)
        cams = (MantisImage * n)(*images)
        out = (MantisResult * rigs)()
        cam_out = (MantisCamResult * n)()
        st = lib().mantis_process_batch(self.h, cams, rigs, n // rigs, out, cam_out)
        self._chk(st, "process_batch")
        return list(out), list(cam_out)

    def process_motion(self, images, delta_pos=None, delta_quat_xyzw=None):
        """mantis_process (one rig) with an optional mantisService motion."""
        n = len(images)
        cams = (MantisImage * n)(*images)
        out = MantisResult()
        cam_out = (MantisCamResult * n)()
        mo = None
        if delta_pos is not None:
            mo = MantisMotion()
            for i in range(3):
                mo.delta_pos[i] = delta_pos[i]
            for i in range(4):
                mo.delta_quat_xyzw[i] = delta_quat_xyzw[i]
        st = lib().mantis_process(self.h, cams, n, None if mo is None else C.byref(mo), C.byref(out), cam_out)
        self._chk(st, "process")
        return out, list(cam_out)

    @property
    def prior_pose(self):
        T = np.zeros((4, 4))
        h = C.c_int32()
        self._chk(lib().mantis_get_prior_pose(self.h, T.ctypes.data, C.byref(h)), "get_prior_pose")
        return T if h.value else None

    @prior_pose.setter
    def prior_pose(self, T):
        if T is None:
            self._chk(lib().mantis_set_prior_pose(self.h, None), "set_prior_pose")
        else:
            T = np.ascontiguousarray(T, np.float64)
            self._chk(lib().mantis_set_prior_pose(self.h, T.ctypes.data), "set_prior_pose")

    def process_sharded(self, images, rigs, cam_index, cams_per_rig):
        """Camera-sharded rig call (mantis_process_rig_sharded): images are this
        rank's cameras cam_index of each rig, rig-major. Returns (rig results,
        every camera's result in global order)."""
        n = len(images)
        n_local = len(cam_index)
        assert n == rigs * n_local
        cams = (MantisImage * n)(*images)
        idx = np.ascontiguousarray(cam_index, np.int32)
        out = (MantisResult * rigs)()
        cam_out = (MantisCamResult * (rigs * cams_per_rig))()
        st = lib().mantis_process_rig_sharded(self.h, cams, rigs, n_local, idx.ctypes.data, cams_per_rig, out, cam_out)
        self._chk(st, "process_rig_sharded")
        return list(out), list(cam_out)

    def shard_gauss_offsets(self, pairs, n_global, gidx, per_frame):
        """k_gauss_offsets_global on gathered (global index, PF flag) pairs
        (mantis_shard_gauss_offsets): (offsets of the local frames gidx, total)."""
        pairs = np.ascontiguousarray(pairs, np.int32).reshape(-1, 2)
        gidx = np.ascontiguousarray(gidx, np.int32)
        off = np.zeros(len(gidx), np.int32)
        tot = C.c_int32()
        self._chk(lib().mantis_shard_gauss_offsets(self.h, pairs.ctypes.data, len(pairs), n_global, gidx.ctypes.data,
                                                   len(gidx), per_frame, off.ctypes.data, C.byref(tot)),
                  "shard_gauss_offsets")
        return off, tot.value

    def comm_info(self):
        nr, rk = C.c_int32(), C.c_int32()
        self._chk(lib().mantis_comm_info(self.h, C.byref(nr), C.byref(rk)), "comm_info")
        return nr.value, rk.value

    def rig_gn(self, rig, cap=4096):
        """(mantis_rig_gn_info, this rank's correspondences [cam, u, v, X, Y, Z])."""
        info = MantisRigGnInfo()
        obs = np.zeros((cap, 6))
        self._chk(lib().mantis_get_rig_gn(self.h, rig, C.byref(info), obs.ctypes.data, cap), "get_rig_gn")
        return info, obs[: min(cap, info.n_obs_local if info.valid else 0)].copy()

    def contours(self, i, max_borders=8192, max_points=1 << 20):
        """Border-following output of frame i of the last batch: a list of
        (points (n, 2) int32, hole) in the library's border order."""
        cnt = np.zeros(max_borders, np.int32)
        hol = np.zeros(max_borders, np.int32)
        pts = np.zeros(2 * max_points, np.int32)
        nb = C.c_int32(0)
        self._chk(lib().mantis_get_contours(self.h, i, cnt.ctypes.data, hol.ctypes.data, max_borders,
                                            pts.ctypes.data, max_points, C.byref(nb)), "get_contours")
        out, k = [], 0
        for b in range(nb.value):
            out.append((pts[2 * k: 2 * (k + cnt[b])].reshape(-1, 2).copy(), int(hol[b])))
            k += int(cnt[b])
        return out

    def frame_counters(self, i):
        out = np.zeros(32, np.int32)
        k = lib().mantis_frame_counters(self.h, i, out.ctypes.data, 32)
        if k < 0:
            raise MantisError("frame_counters: bad frame index")
        return out[:k]

    def frame_debug(self, i):
        d = FrameDebug()
        assert C.sizeof(d) == lib().mantis_frame_debug_size(), "FrameDebug layout mismatch"
        self._chk(lib().mantis_get_frame_debug(self.h, i, C.byref(d), C.sizeof(d)), "get_frame_debug")
        return d

    def canny(self, img):
        out = np.zeros((img.height, img.width), np.uint8)
        self._chk(lib().mantis_canny(self.h, C.byref(img), out.ctypes.data), "canny")
        return out

    def hysteresis(self, cls):
        """cv::Canny's hysteresis on a class plane (0 none, 1 weak candidate, 2 strong)."""
        cls = np.ascontiguousarray(cls, np.uint8)
        h, w = cls.shape
        out = np.zeros((h, w), np.uint8)
        self._chk(lib().mantis_hysteresis(self.h, cls.ctypes.data, w, h, out.ctypes.data), "hysteresis")
        return out

    def masks(self, img):
        det = np.zeros((img.height, img.width), np.uint8)
        mask = np.zeros((img.height, img.width), np.uint8)
        self._chk(lib().mantis_masks(self.h, C.byref(img), det.ctypes.data, mask.ctypes.data), "masks")
        return det, mask

    def detect_quads(self, img, max_quads=256):
        corners = np.zeros((max_quads, 8), np.int32)
        n = C.c_int32()
        self._chk(lib().mantis_detect_quads(self.h, C.byref(img), corners.ctypes.data, max_quads, C.byref(n)),
                  "detect_quads")
        return corners[: n.value].copy()

    def score(self, img, c2w, fast=True, mask=None):
        c2w = np.ascontiguousarray(c2w, np.float64).reshape(-1, 12)
        n = len(c2w)
        err = np.zeros(n)
        npj = np.zeros(n, np.int32)
        mptr = None
        if mask is not None:
            mask = np.ascontiguousarray(mask, np.uint8)
            mptr = mask.ctypes.data
        self._chk(lib().mantis_score_hypotheses(self.h, C.byref(img), mptr, c2w.ctypes.data, n, int(fast),
                                                err.ctypes.data, npj.ctypes.data), "score_hypotheses")
        return err, npj

    def comm_init(self, rank, world, dist=None):
        """RCCL communicator for this context: rank 0 creates the unique id and
        torch.distributed (any backend) broadcasts it."""
        uid = (C.c_uint8 * 128)()
        if rank == 0:
            self._chk(lib().mantis_comm_unique_id(uid), "comm_unique_id")
        if dist is not None and world > 1:
            box = [bytes(uid)]
            dist.broadcast_object_list(box, src=0)
            C.memmove(uid, box[0], 128)
        self._chk(lib().mantis_comm_init(self.h, uid, world, rank), "comm_init")

    def score_argmin(self, img, c2w, index_base=0, use_comm=False, mask=None):
        """Dense scoring + first-minimum argmin (config 5); returns (err, global index)."""
        c2w = np.ascontiguousarray(c2w, np.float64).reshape(-1, 12)
        e = C.c_double()
        i = C.c_int64()
        mk = None if mask is None else np.ascontiguousarray(mask, np.uint8)
        self._chk(lib().mantis_score_argmin(self.h, C.byref(img), None if mk is None else mk.ctypes.data,
                                            c2w.ctypes.data, len(c2w), index_base, int(use_comm), C.byref(e),
                                            C.byref(i)), "score_argmin")
        return e.value, i.value

    def score_argmin_dev(self, img, c2w_dev, n, index_base=0, use_comm=False, mask_dev=None):
        """score_argmin on device-resident inputs (mantis_score_argmin_dev): c2w_dev = device
        pointer to n x 12 doubles, mask_dev = device pointer to W*H bytes or None."""
        e = C.c_double()
        i = C.c_int64()
        self._chk(lib().mantis_score_argmin_dev(self.h, C.byref(img), None if mask_dev is None else C.c_void_p(mask_dev),
                                                C.c_void_p(c2w_dev), int(n), index_base, int(use_comm), C.byref(e),
                                                C.byref(i)), "score_argmin_dev")
        return e.value, i.value

    def score_argmin_batch(self, imgs, c2w_devs, ns, index_bases=None, use_comm=False, mask_devs=None):
        """mantis_score_argmin_batch: per-frame device hypothesis blocks (and
        masks) scored in one launch; returns [(err, global index)] per frame."""
        nf = len(imgs)
        arr = (MantisImage * nf)(*imgs)
        cp = (C.c_void_p * nf)(*[C.c_void_p(p) for p in c2w_devs])
        mp = None if mask_devs is None else (C.c_void_p * nf)(*[C.c_void_p(p) for p in mask_devs])
        n = np.ascontiguousarray(ns, np.int32)
        ib = np.ascontiguousarray(index_bases if index_bases is not None else np.zeros(nf), np.int64)
        e = np.zeros(nf)
        i = np.zeros(nf, np.int64)
        self._chk(lib().mantis_score_argmin_batch(self.h, arr, nf, mp, cp, n.ctypes.data, ib.ctypes.data,
                                                  int(use_comm), e.ctypes.data, i.ctypes.data), "score_argmin_batch")
        return list(zip(e.tolist(), i.tolist()))

    def rpp(self, img_pts, obj_pts):
        img_pts = np.ascontiguousarray(img_pts, np.float64).reshape(-1, 4, 2)
        obj_pts = np.ascontiguousarray(obj_pts, np.float64).reshape(-1, 4, 3)
        n = len(img_pts)
        R = np.zeros((n, 9))
        t = np.zeros((n, 3))
        e = np.zeros((n, 2))
        s = np.zeros(n, np.int32)
        self._chk(lib().mantis_rpp_batch(self.h, img_pts.ctypes.data, obj_pts.ctypes.data, n, R.ctypes.data,
                                         t.ctypes.data, e.ctypes.data, s.ctypes.data), "rpp_batch")
        return R.reshape(n, 3, 3), t, e, s

    def rpp_solve(self, model, iprts):
        """RPP::Rpp(model, iprts) (RPP.cpp:13-64) on the device for any point
        count 4..12 (mantis_rpp_solve): model 3 x n (or k x 3 x n), iprts 3 x n
        homogeneous with a unit third row (demo.cpp:41-53's layout). Returns
        (R [k,3,3], t [k,3], errs [k,2] = obj_err, img_err, status [k], iterations [k])."""
        m = np.asarray(model, np.float64)
        q = np.asarray(iprts, np.float64)
        if m.ndim == 2:
            m, q = m[None], q[None]
        k, _, npts = m.shape
        if not np.all(q[:, 2, :] == 1.0):
            raise ValueError("rpp_solve: image points must be homogeneous with z = 1")
        obj = np.ascontiguousarray(np.transpose(m, (0, 2, 1)))      # k x n x 3
        img = np.ascontiguousarray(np.transpose(q[:, :2, :], (0, 2, 1)))  # k x n x 2
        R = np.zeros((k, 9))
        t = np.zeros((k, 3))
        e = np.zeros((k, 2))
        s = np.zeros(k, np.int32)
        it = np.zeros(k, np.int32)
        self._chk(lib().mantis_rpp_solve(self.h, img.ctypes.data, obj.ctypes.data, int(npts), int(k), R.ctypes.data,
                                         t.ctypes.data, e.ctypes.data, s.ctypes.data, it.ctypes.data), "rpp_solve")
        return R.reshape(k, 3, 3), t, e, s, it

    def rig_weights(self, rig, cams_per_rig=None):
        """Legacy rig weighting record of rig `rig` (mantis_get_rig_weights):
        (weights[C+1], c2w[C+1, C, 12], sums[C+1, C, 2], chosen slot or -1);
        slot C = the mantisService motion prediction. The buffers are sized from
        the record's own camera count (mantis_get_rig_weights_info); a
        cams_per_rig that disagrees with it is an error."""
        rigs, Cn = C.c_int32(), C.c_int32()
        self._chk(lib().mantis_get_rig_weights_info(self.h, C.byref(rigs), C.byref(Cn)), "get_rig_weights_info")
        Cn = Cn.value
        if cams_per_rig is not None and cams_per_rig != Cn:
            raise MantisError(f"rig_weights: the last batch had {Cn} cameras per rig, not {cams_per_rig}")
        w = np.zeros(Cn + 1)
        c2w = np.zeros((Cn + 1, Cn, 12))
        sums = np.zeros((Cn + 1, Cn, 2))
        ch = C.c_int32()
        self._chk(lib().mantis_get_rig_weights(self.h, rig, w.ctypes.data, c2w.ctypes.data, sums.ctypes.data,
                                               C.byref(ch)), "get_rig_weights")
        return w, c2w, sums, ch.value

    # Markov yaw filter (include/mantis3/Markov.cpp) ----------------------
    def markov_init(self, w2c_R):
        R = np.ascontiguousarray(w2c_R, np.float64).reshape(-1, 9)
        self._markov_n = len(R)
        self._chk(lib().mantis_markov_init(self.h, len(R), R.ctypes.data), "markov_init")

    def _markov_len(self, arr, what):
        n = getattr(self, "_markov_n", None)
        if n is None:
            raise MantisError("markov: no filters (markov_init first)")
        if len(arr) != n:  # the C API reads markov_n entries of each array
            raise MantisError(f"markov: {what} has {len(arr)} entries, the context holds {n} filters")

    def markov_sense(self, w2c_R, active=None):
        R = np.ascontiguousarray(w2c_R, np.float64).reshape(-1, 9)
        a = None if active is None else np.ascontiguousarray(active, np.int32)
        self._markov_len(R, "w2c_R")
        if a is not None:
            self._markov_len(a, "active")
        self._chk(lib().mantis_markov_sense(self.h, R.ctypes.data, None if a is None else a.ctypes.data),
                  "markov_sense")

    def markov_convolve(self, dtheta, dt, active=None):
        th = np.ascontiguousarray(dtheta, np.float64)
        d = np.ascontiguousarray(dt, np.float64)
        a = None if active is None else np.ascontiguousarray(active, np.int32)
        self._markov_len(th, "dtheta")
        self._markov_len(d, "dt")
        if a is not None:
            self._markov_len(a, "active")
        self._chk(lib().mantis_markov_convolve(self.h, th.ctypes.data, d.ctypes.data,
                                               None if a is None else a.ctypes.data), "markov_convolve")

    def markov_weight(self, f, w2c_R, error):
        R = np.ascontiguousarray(w2c_R, np.float64).reshape(-1, 9)
        e = np.ascontiguousarray(error, np.float64).copy()
        self._chk(lib().mantis_markov_weight(self.h, f, R.ctypes.data, len(R), e.ctypes.data), "markov_weight")
        return e

    def markov_get(self):
        n = self._markov_n
        planes = np.zeros((n, 360))
        yaw = np.zeros(n)
        am = np.zeros(n, np.int32)
        self._chk(lib().mantis_markov_get(self.h, planes.ctypes.data, yaw.ctypes.data, am.ctypes.data), "markov_get")
        return planes, yaw, am

    def quad_gn(self, img_pts, obj_pts, R, t, iterations):
        """Per-quad GN after RPP (mantis_quad_gn): (R, t, steps, costs)."""
        img_pts = np.ascontiguousarray(img_pts, np.float64).reshape(-1, 4, 2)
        obj_pts = np.ascontiguousarray(obj_pts, np.float64).reshape(-1, 4, 3)
        n = len(img_pts)
        R = np.ascontiguousarray(R, np.float64).reshape(n, 9).copy()
        t = np.ascontiguousarray(t, np.float64).reshape(n, 3).copy()
        steps = np.zeros(n, np.int32)
        costs = np.zeros((n, 2))
        self._chk(lib().mantis_quad_gn(self.h, img_pts.ctypes.data, obj_pts.ctypes.data, n, R.ctypes.data,
                                       t.ctypes.data, iterations, steps.ctypes.data, costs.ctypes.data), "quad_gn")
        return R.reshape(n, 3, 3), t, steps, costs

    # device buffers -------------------------------------------------------
    def device_alloc(self, nbytes):
        p = C.c_void_p()
        self._chk(lib().mantis_device_alloc(self.h, nbytes, C.byref(p)), "device_alloc")
        return p.value

    def device_free(self, p):
        self._chk(lib().mantis_device_free(self.h, C.c_void_p(p)), "device_free")

    def h2d(self, dst, arr):
        arr = np.ascontiguousarray(arr)
        self._chk(lib().mantis_memcpy_h2d(self.h, C.c_void_p(dst), arr.ctypes.data, arr.nbytes), "h2d")

    def d2h(self, arr, src):
        self._chk(lib().mantis_memcpy_d2h(self.h, arr.ctypes.data, C.c_void_p(src), arr.nbytes), "d2h")
        return arr

    def synth_render(self, cams, seeds, out_dev):
        n = len(cams)
        arr = (SynthCamC * n)()
        for i, c in enumerate(cams):
            C.memmove(C.byref(arr[i]), C.byref(c), C.sizeof(SynthCamC))
        s = np.ascontiguousarray(seeds, np.uint64)
        self._chk(lib().mantis_synth_render(self.h, arr, n, s.ctypes.data, C.c_void_p(out_dev)), "synth_render")

    def synchronize(self):
        self._chk(lib().mantis_synchronize(self.h), "synchronize")

    def set_profiling(self, on):
        self._chk(lib().mantis_set_profiling(self.h, int(on)), "set_profiling")

    def kernel_times(self):
        names = (C.c_char_p * 64)()
        ms = (C.c_float * 64)()
        n = lib().mantis_kernel_times(self.h, names, ms, 64)
        return [(names[i].decode(), ms[i]) for i in range(n)]

    def stage_times(self):
        """kernel_times() summed per stage: a mark named "stage/kernel" (the
        hot stages are marked per kernel) counts toward "stage"."""
        out = {}
        for name, ms in self.kernel_times():
            st = name.split("/", 1)[0]
            out[st] = out.get(st, 0.0) + ms
        return list(out.items())


def argmin_pick(pairs):
    """The cross-shard first-minimum rule of mantis_score_argmin (host only):
    pairs = ranks x (err, global index), index -1 for an empty shard."""
    pairs = np.ascontiguousarray(pairs, np.float64).reshape(-1, 2)
    e = C.c_double()
    i = C.c_int64()
    st = lib().mantis_argmin_pick(pairs.ctypes.data, len(pairs), C.byref(e), C.byref(i))
    if st != MANTIS_OK:
        raise MantisError(f"argmin_pick failed ({st})")
    return e.value, i.value
