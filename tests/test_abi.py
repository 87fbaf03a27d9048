"""The drop-in boundary: libmantis_amd.so loads on a CPU-only host, exports
every entry point include/mantis.h and include/mantis_ros.h declare, and its host-only functions
(defaults, map parsing, the 6x6 GN solve, error paths) behave. No compute
calls are made without a GPU.
"""
import ctypes as C
import os
import re

import numpy as np
import pytest

import _gn_ref as G
import _oracle as O

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADERS = [os.path.join(ROOT, "include", h) for h in ("mantis.h", "mantis_ros.h")]


def _declared():
    names = set()
    for h in HEADERS:
        src = re.sub(r"/\*.*?\*/", "", open(h).read(), flags=re.S)
        names |= set(re.findall(r"\b(mantis_[a-z0-9_]+)\s*\(", src))
    return sorted(names)


def test_library_exports_every_declared_symbol():
    import mantis_amd as M

    L = M.lib()
    names = _declared()
    assert len(names) >= 30
    missing = [n for n in names if not hasattr(L, n)]
    assert not missing, missing
    # and the Python mirror binds every one of them
    assert set(names) <= set(M._SIGS), sorted(set(names) - set(M._SIGS))


def test_default_config_and_abi_version():
    import mantis_amd as M

    cfg = M.default_config()
    assert cfg.struct_size == C.sizeof(M.MantisConfig)
    assert (cfg.particles, cfg.iterations, cfg.canny_low, cfg.polygon_epsilon) == (50, 10, 50, 10.0)
    assert cfg.rng_seed == 1 and cfg.gn_enable == 0
    assert M.lib().mantis_abi_version() >= 1


def test_parse_coordinates_matches_oracle():
    import yaml

    import mantis_amd as M

    y = yaml.safe_load(open(os.path.join(ROOT, "tests", "golden", "map.yaml")))
    for key in ("whiteMap", "redMap", "greenMap"):
        s = y[key].encode()
        buf = np.zeros(3 * 4096)
        n = M.lib().mantis_parse_coordinates(s, buf.ctypes.data, 4096)
        assert np.array_equal(buf[: 3 * n].reshape(n, 3), O.parse_coordinates(y[key]))


def test_gn_solve_matches_numpy():
    import mantis_amd as M

    rng = np.random.default_rng(2)
    T = np.eye(4)
    T[:3, 3] = [0.3, -0.2, 1.5]
    ext = [np.eye(4) for _ in range(3)]
    for c in range(3):
        ext[c][:3, 3] = [0.1 * c, 0, 0]
    obs = G.synth_rig_obs(rng, T, ext)
    acc = G.gn_accumulate(T @ G.exp_se3_right(np.eye(4), np.array([0.01, -0.02, 0.01, 0.02, 0.0, -0.01])), ext, obs)
    T0 = np.ascontiguousarray(np.eye(4))
    Tc = T0.copy()
    d6 = np.zeros(6)
    st = M.lib().mantis_gn_solve(np.ascontiguousarray(acc).ctypes.data, 1e-9, Tc.ctypes.data, d6.ctypes.data)
    assert st == 0
    Tn, x = G.gn_solve(acc, 1e-9, T0)
    np.testing.assert_allclose(d6, x, rtol=1e-10, atol=1e-13)
    np.testing.assert_allclose(Tc, Tn, rtol=0, atol=1e-12)
    # not positive definite -> argument error, T untouched
    Tz = np.eye(4)
    assert M.lib().mantis_gn_solve(np.zeros(28).ctypes.data, 0.0, Tz.ctypes.data, None) == 1
    assert np.array_equal(Tz, np.eye(4))


def test_null_arguments_rejected():
    import mantis_amd as M

    L = M.lib()
    assert L.mantis_destroy(None) == 1
    assert L.mantis_rng_set(None, 5) == 1
    assert L.mantis_process(None, None, 0, None, None, None) == 1


def _has_gpu():
    try:
        import torch

        return torch.cuda.device_count() > 0
    except Exception:
        return False


@pytest.mark.skipif(_has_gpu(), reason="error path for hosts without a GPU")
def test_create_without_gpu_fails_loudly():
    import mantis_amd as M

    cfg = M.default_config()
    h = C.c_void_p()
    st = M.lib().mantis_create(C.byref(cfg), C.byref(h))
    assert st == 2 and not h.value
    msg = M.lib().mantis_last_error(None)
    assert msg and b"GPU" in msg
    with pytest.raises(M.MantisError):
        M.Mantis()


def test_create_rejects_oversized_frames():
    """Hysteresis run ids and their band row share a list word: configs past
    2^25 pixels are refused at creation (before any device call, so this runs
    without a GPU too)."""
    import mantis_amd as M

    cfg = M.default_config()
    cfg.max_width, cfg.max_height = 8190, 4200
    h = C.c_void_p()
    st = M.lib().mantis_create(C.byref(cfg), C.byref(h))
    assert st == 1 and not h.value  # MANTIS_ERR_ARG
    assert b"2^25" in M.lib().mantis_last_error(None)


def test_create_rejects_tall_frames():
    """Border walks (Walk.pos) and the contour pool (PtPacked) pack a padded
    row index in 16 bits: heights past 65533 are refused at creation (before
    any device call)."""
    import mantis_amd as M

    cfg = M.default_config()
    cfg.max_width, cfg.max_height = 16, 70000  # 1.1 M pixels: inside the 2^25 bound
    h = C.c_void_p()
    st = M.lib().mantis_create(C.byref(cfg), C.byref(h))
    assert st == 1 and not h.value  # MANTIS_ERR_ARG
    assert b"65533" in M.lib().mantis_last_error(None)
