"""Markov yaw filter (include/mantis3/Markov.cpp MarkovModel).

CPU: the oracle restatement (oracle/o_markov.cpp) against an independent
numpy form of updateWeights (a circular discrete Gaussian over the 360 bins,
normalized) and the reference's quirks (convolve truncates dTheta to whole
radians before converting to degrees, getYaw returns p[argmax] * pi / 180).
The reference holds no tests or fixtures for this class: parity unpinned
against the reference itself.
GPU: the library's planes (mantis_markov_*) bit-identical to the oracle's
through a sequence of init / sense / convolve / weight operations.
"""
import math

import numpy as np
import pytest

import _oracle as O
from mantis_amd import synth


def _yaw_R(deg):
    """A w2c basis whose getRPY yaw is `deg` (camera looking down, slight tilt)."""
    return (synth.rot_z(math.radians(deg)) @ synth.rot_y(0.1) @ synth.rot_x(0.05)).reshape(9)


def _np_update(y, stddev):
    """updateWeights as a circular Gaussian: mu_j is the representative of j
    within (i - 180, i + 180] the reference's loops pick."""
    out = np.zeros(360)
    den = stddev * math.sqrt(2 * math.pi)
    for i in range(360):
        j = np.arange(360)
        d = i - j
        d = np.where(d > 180, d - 360, np.where(d < -179, d + 360, d))
        out[i] = np.sum((y / den) * np.exp(-(d * d) / (2 * stddev * stddev)))
    return out / out.sum()


def test_markov_oracle_against_numpy_and_quirks():
    b = O.Markov.bin(_yaw_R(37.4))
    assert b == 37
    m = O.Markov(_yaw_R(37.4))
    one = np.zeros(360)
    one[37] = 1
    np.testing.assert_allclose(m.p, _np_update(one, 3.0), rtol=1e-12, atol=1e-300)
    assert abs(m.p.sum() - 1) < 1e-14 and int(np.argmax(m.p)) == 37
    y, am = m.yaw()
    assert am == 37 and y == m.p[37] * math.pi / 180  # getYaw's return value (quirk)
    # sense at the same yaw sharpens the peak
    p0 = m.p.copy()
    m.sense(_yaw_R(37.9))
    sense = _np_update(one, 3.5)
    ref = p0 * sense
    np.testing.assert_allclose(m.p, ref / ref.sum(), rtol=1e-12, atol=1e-300)
    assert m.p[37] > p0[37]
    # convolve: 0.9 rad truncates to 0 -> blur only; 2.5 rad -> (int)2 * 180 / pi = 114 bins
    m2 = O.Markov(_yaw_R(100.2))
    q = m2.p.copy()
    m2.convolve(0.9, 30.0)
    np.testing.assert_allclose(m2.p, _np_update(q, 11.5 / 3.0 / 1.0 * 30.0 / 30.0), rtol=1e-12, atol=1e-300)
    assert int(np.argmax(m2.p)) == 100
    m2.convolve(2.5, 30.0)
    assert int(np.argmax(m2.p)) == 214
    m2.convolve(-2.5, 30.0)
    assert int(np.argmax(m2.p)) == 100
    m2.convolve(-7.2, 30.0)  # (int)-7 * 180 / pi = -401 bins: 41 bins back
    assert int(np.argmax(m2.p)) == 59
    # updateHypothesis: error / p[bin]
    R = np.array([_yaw_R(a) for a in (59.5, 10.0, 300.0)])
    e = m2.weight(R, [2.0, 3.0, 5.0])
    assert e[0] == 2.0 * 1 / m2.p[59] and e[1] == 3.0 * 1 / m2.p[10] and e[2] == 5.0 * 1 / m2.p[300]


@pytest.mark.gpu
def test_markov_device_bit_identical_to_oracle():
    import mantis_amd as M

    rng = np.random.default_rng(9)
    n = 16
    yaws = rng.uniform(0, 360, n)
    R0 = np.array([_yaw_R(a) for a in yaws])
    m = M.Mantis(max_cams=1)
    m.markov_init(R0)
    orc = [O.Markov(R0[f]) for f in range(n)]
    planes, yaw, am = m.markov_get()
    for f in range(n):
        assert np.array_equal(planes[f], orc[f].p), f
    for step in range(4):
        Rs = np.array([_yaw_R(a + rng.normal() * 3) for a in yaws])
        active = (rng.uniform(size=n) < 0.8).astype(np.int32)
        m.markov_sense(Rs, active)
        for f in range(n):
            if active[f]:
                orc[f].sense(Rs[f])
        dth = rng.uniform(-8, 8, n)
        dt = rng.uniform(0.5, 40, n)
        m.markov_convolve(dth, dt)
        for f in range(n):
            orc[f].convolve(dth[f], dt[f])
        planes, yaw, am = m.markov_get()
        for f in range(n):
            assert np.array_equal(planes[f], orc[f].p), (step, f)
            oy, oam = orc[f].yaw()
            assert yaw[f] == oy and am[f] == oam
    Rh = np.array([_yaw_R(a) for a in rng.uniform(0, 360, 40)])
    err = rng.uniform(1e3, 1e5, 40)
    for f in (0, 7, 15):
        assert np.array_equal(m.markov_weight(f, Rh, err), orc[f].weight(Rh, err))
    m.close()
