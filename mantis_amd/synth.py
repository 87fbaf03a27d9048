"""Synthetic inputs for tests and the bench.

Camera model: the fisheye K/D of test/unit_test.cpp:144-145 (1280x1024
camera), re-centred for 1280x720 (cy = 501.5538330078125 - 152) and scaled
x1.5 for 1920x1080.  Poses: camera height U[1, 2] m, tilt <= 25 deg, yaw
U[0, 2pi), x, y U[-0.48, 0.48], from a seeded numpy Generator.  4-camera rig
(config 3): cameras yawed 0/90/180/270 deg about base Z, tilted 20 deg
outward, offset 0.1 m from the base origin.

Rendering runs either on the host (tools/libmantis_synth.so, CPU tests) or in
HBM through the product library's HIP kernel (bench).  Both evaluate
mantis_amd/csrc/synth.h.
"""
import ctypes as C
import math
import os

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SYNTH_SO = os.path.join(ROOT, "tools", "libmantis_synth.so")

FX, FY = 323.1511535644531, 322.78955078125
D_FISHEYE = np.array([0.0029509200248867273, -0.009944040328264236, 0.005587350111454725, -0.00205406011082232])
SEED_BASE = 0x4D414E5449530000


class SynthCam(C.Structure):
    _fields_ = [("fx", C.c_double), ("fy", C.c_double), ("cx", C.c_double), ("cy", C.c_double),
                ("k", C.c_double * 4), ("R_wc", C.c_double * 9), ("pos", C.c_double * 3),
                ("w", C.c_int32), ("h", C.c_int32), ("pad", C.c_int32 * 2)]


def intrinsics(w=1280, h=720):
    """K (3x3) and D (4,) for the named resolution."""
    if (w, h) == (1280, 720):
        K = np.array([[FX, 0, 642.658203125], [0, FY, 349.5538330078125], [0, 0, 1.0]])
    elif (w, h) == (1920, 1080):
        K = np.array([[FX * 1.5, 0, 642.658203125 * 1.5], [0, FY * 1.5, 349.5538330078125 * 1.5], [0, 0, 1.0]])
    else:
        K = np.array([[FX * w / 1280.0, 0, w / 2.0], [0, FY * w / 1280.0, h / 2.0], [0, 0, 1.0]])
    return K, D_FISHEYE.copy()


def rot_x(a):
    c, s = math.cos(a), math.sin(a)
    return np.array([[1, 0, 0], [0, c, -s], [0, s, c]])


def rot_y(a):
    c, s = math.cos(a), math.sin(a)
    return np.array([[c, 0, s], [0, 1, 0], [-s, 0, c]])


def rot_z(a):
    c, s = math.cos(a), math.sin(a)
    return np.array([[c, -s, 0], [s, c, 0], [0, 0, 1]])


NADIR = np.array([[1.0, 0, 0], [0, -1.0, 0], [0, 0, -1.0]])  # camera x right, y down, z = -Z_world


def random_pose(rng):
    """(R_wc, pos): camera-to-world rotation and camera centre."""
    h = rng.uniform(1.0, 2.0)
    yaw = rng.uniform(0, 2 * math.pi)
    tilt = math.radians(25.0) * math.sqrt(rng.uniform(0, 1))
    tdir = rng.uniform(0, 2 * math.pi)
    R = rot_z(yaw) @ NADIR @ rot_x(tilt * math.cos(tdir)) @ rot_y(tilt * math.sin(tdir))
    pos = np.array([rng.uniform(-0.48, 0.48), rng.uniform(-0.48, 0.48), h])
    return R, pos


def rig_extrinsics(n_cams=4, tilt_deg=20.0, offset=0.1):
    """T_base_cam (4x4) for an n-camera ring: yaw 360/n apart, tilted outward."""
    out = []
    for i in range(n_cams):
        yaw = 2 * math.pi * i / n_cams
        R = rot_z(yaw) @ NADIR @ rot_y(-math.radians(tilt_deg))
        T = np.eye(4)
        T[:3, :3] = R
        T[:3, 3] = rot_z(yaw) @ np.array([offset, 0.0, 0.0])
        out.append(T)
    return out


def random_base_pose(rng):
    h = rng.uniform(1.0, 2.0)
    yaw = rng.uniform(0, 2 * math.pi)
    tilt = math.radians(10.0) * math.sqrt(rng.uniform(0, 1))
    tdir = rng.uniform(0, 2 * math.pi)
    R = rot_z(yaw) @ rot_x(tilt * math.cos(tdir)) @ rot_y(tilt * math.sin(tdir))
    T = np.eye(4)
    T[:3, :3] = R
    T[:3, 3] = [rng.uniform(-0.48, 0.48), rng.uniform(-0.48, 0.48), h]
    return T


def make_cam(R_wc, pos, w=1280, h=720):
    K, D = intrinsics(w, h)
    c = SynthCam()
    c.fx, c.fy, c.cx, c.cy = K[0, 0], K[1, 1], K[0, 2], K[1, 2]
    for i in range(4):
        c.k[i] = D[i]
    R = np.asarray(R_wc, np.float64).reshape(9)
    for i in range(9):
        c.R_wc[i] = R[i]
    for i in range(3):
        c.pos[i] = pos[i]
    c.w, c.h = w, h
    return c


def frame_seed(cfg, frame):
    return (SEED_BASE + cfg * 1000003 + frame) & 0xFFFFFFFFFFFFFFFF


_lib = None


def _host_lib():
    global _lib
    if _lib is None:
        if not os.path.exists(SYNTH_SO):
            raise RuntimeError("tools/libmantis_synth.so not built (run __graft_entry__.build())")
        _lib = C.CDLL(SYNTH_SO)
        _lib.mantis_synth_render_host.argtypes = [C.POINTER(SynthCam), C.c_uint64, C.c_void_p]
    return _lib


def render_host(cam, seed):
    out = np.zeros((cam.h, cam.w, 3), np.uint8)
    _host_lib().mantis_synth_render_host(C.byref(cam), C.c_uint64(seed), out.ctypes.data)
    return out


def truth_c2w(R_wc, pos):
    """Reference-convention c2w (world -> camera) as 12 doubles (R row-major, t)."""
    R = np.asarray(R_wc).T
    t = -R @ np.asarray(pos)
    return np.concatenate([R.reshape(9), t])


def load_map(path=None):
    """(white, red, green) landmark arrays from the committed map fixture (params/map.yaml data)."""
    if path is None:
        path = os.path.join(ROOT, "tests", "golden", "map.yaml")
    import yaml

    with open(path) as f:
        d = yaml.safe_load(f)

    def parse(s):
        # std::getline(';') semantics (Mantis3Params.h:132): no row after a final ';'
        raw = s.split(";")
        if raw and raw[-1] == "":
            raw.pop()
        rows = [r.replace("\n", "").replace(" ", "") for r in raw]
        out = []
        for r in rows:
            parts = (r.split(",") + ["", "", ""])[:3]
            vals = []
            for p in parts:
                try:
                    vals.append(float(p))
                except ValueError:
                    vals.append(0.0)
            out.append(vals)
        return np.array(out, np.float64)

    return parse(d["whiteMap"]), parse(d["redMap"]), parse(d["greenMap"])
