#!/usr/bin/env python3
"""Generate the committed golden fixtures under tests/golden/.

Run in the build container (it needs /root/reference for the in-place
Rpoly.cpp build and for test/grid1.jpg):

    make oracle ref && python tests/golden/make_golden.py

Fixtures (data only — inputs and expected outputs):
  rpp_golden.npz    4-point RPP problems -> outputs of the ORACLE's RPP
                    restatement (oracle/o_rpp.cpp; RPP.cpp itself needs
                    OpenCV and is unbuildable here, so these are regression
                    fixtures: the RPP pin is demo.cpp's known answer). Cases:
                    test/unit_test.cpp:144-203 (fisheye PnP, cv::RNG(10)
                    sigma 0.01 corner noise, GCC right-to-left draw order),
                    test/legacy/unit_test.cpp:49-76 (pinhole square), and
                    seeded random squares seen by a nadir-ish camera.
  rpp_faults.npz    degenerate 4-point RPP problems -> the ORACLE's outputs
                    (regression fixtures, as above): image points whose mean ray is the optical
                    axis (a centred symmetric square), collinear, pairwise
                    repeated and coincident points -- Rpp() returns false there
                    (no 2nd-pose candidate: DecomposeR / RpyAng_X fail,
                    RPP.cpp:13-64, 755-808), status 0 -- plus tiny / huge
                    spreads that still succeed. (The exit(1) of
                    GetRotationbyVector, RPP.cpp:450-453, needs a mean ray the
                    rotation cannot map back; no image points with z = 1 reach
                    it -- tests/test_oracle_pins.py searches for it.)
  rpp_demo.npz      demo.cpp:17-38 10-point problem -> the oracle's output
                    plus the Matlab answer quoted in demo.cpp:28-38 (the pin).
  rpoly_golden.npz  quartics -> the REFERENCE's own rpoly_ak1 roots (5 slots;
                    Rpoly.cpp compiled in place, oracle/_ref/libref_rpoly.so).
  grid1.npz         test/grid1.jpg decoded to BGR (PIL) + config-1 K/D, and
                    the ORACLE's quad corners / publish decision for it
                    (a plumbing golden: the reference itself cannot run here).
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

import _oracle as O  # noqa: E402
from mantis_amd import synth  # noqa: E402

REF_GRID1 = "/root/reference/test/grid1.jpg"


def rodrigues(rv):
    rv = np.asarray(rv, float)
    th = np.linalg.norm(rv)
    k = rv / th
    Kx = np.array([[0, -k[2], k[1]], [k[2], 0, -k[0]], [-k[1], k[0], 0]])
    return np.eye(3) + np.sin(th) * Kx + (1 - np.cos(th)) * Kx @ Kx


def ref_case(model, ip):
    st, R, t, e, _code = O.rpp(model, ip)
    return st, R, t, e


def rpp_cases():
    models, iprts, names = [], [], []
    # test/unit_test.cpp:144-203
    R = rodrigues([0.8, np.pi, 0.6])
    tv = np.array([0, 0.7, 1.0])
    obj = np.array([[0.155, 0.155, 0], [-0.155, 0.155, 0], [-0.155, -0.155, 0], [0.155, -0.155, 0]])
    g, _ = O.gaussians(10, 8)  # cv::RNG(10) stream
    noise = np.asarray(g, np.float64) * 0.01
    ip = np.ones((3, 4))
    for k in range(4):
        # tf::Vector3(rng.gaussian(), rng.gaussian(), 0): GCC draws the 2nd argument first
        p = obj[k] + np.array([noise[2 * k + 1], noise[2 * k], 0.0])
        q = R @ p + tv
        ip[0, k], ip[1, k] = q[0] / q[2], q[1] / q[2]
    models.append(obj.T.copy())
    iprts.append(ip)
    names.append("unit_test.cpp:144-203")
    # test/legacy/unit_test.cpp:49-76 (second case, noiseless pinhole square)
    R = rodrigues([-1, np.pi, 0])
    tv = np.array([0, 0.6, 3.0])
    obj = np.array([[0.5, 0.5, 0], [-0.5, 0.5, 0], [-0.5, -0.5, 0], [0.5, -0.5, 0]])
    q = (R @ obj.T) + tv[:, None]
    models.append(obj.T.copy())
    iprts.append(np.vstack([q[0] / q[2], q[1] / q[2], np.ones(4)]))
    names.append("legacy/unit_test.cpp:49-76")
    # seeded random squares (the detector's +-0.16 model, both orientations)
    rng = np.random.default_rng(20261015)
    s = 0.16
    sq = [np.array([[s, -s, -s, s], [s, s, -s, -s], [0, 0, 0, 0.0]]),
          np.array([[s, -s, -s, s], [-s, -s, s, s], [0, 0, 0, 0.0]])]
    for k in range(400):
        tilt = 0.3 if k < 300 else 1.4
        R = synth.rot_z(rng.uniform(0, 2 * np.pi)) @ synth.NADIR @ synth.rot_x(rng.normal() * tilt)
        t = np.array([rng.normal() * 0.3, rng.normal() * 0.3, rng.uniform(0.8, 3.0)])
        m = sq[k % 2]
        Q = R.T @ m + t[:, None]
        ip = np.vstack([Q[0] / Q[2], Q[1] / Q[2], np.ones(4)])
        ip[:2] += rng.normal(size=(2, 4)) * (0.003 if k % 3 else 0.03)
        models.append(m.copy())
        iprts.append(ip)
        names.append(f"random[{k}]")
    out = {"model": np.array(models), "iprts": np.array(iprts), "name": np.array(names)}
    st, Rs, ts, es = [], [], [], []
    for m, ip in zip(models, iprts):
        a, R, t, e = ref_case(m, ip)
        st.append(a)
        Rs.append(R)
        ts.append(t)
        es.append(e)
    out.update(status=np.array(st, np.int32), R=np.array(Rs), t=np.array(ts), errs=np.array(es))
    return out


def rpp_fault_cases():
    rng = np.random.default_rng(20261017)
    s = 0.16
    sq = np.array([[s, -s, -s, s], [s, s, -s, -s], [0, 0, 0, 0.0]])
    models, iprts, names = [], [], []

    def add(name, ip, m=sq):
        models.append(m.copy())
        iprts.append(np.asarray(ip, np.float64))
        names.append(name)

    for k in range(12):
        a = rng.uniform(0.05, 0.6)
        add(f"centred_square[{k}]", [[a, -a, -a, a], [a, a, -a, -a], [1, 1, 1, 1]])
    for k in range(12):
        d, o, tt = rng.normal(size=2), rng.normal(size=2) * 0.3, np.sort(rng.uniform(-1, 1, 4))
        add(f"collinear[{k}]", [o[0] + d[0] * tt, o[1] + d[1] * tt, np.ones(4)])
    for k in range(12):
        p = rng.normal(size=(2, 4)) * 0.3
        p[:, 1], p[:, 3] = p[:, 0], p[:, 2]
        add(f"repeated[{k}]", np.vstack([p, np.ones(4)]))
    for k in range(6):
        p = rng.normal(size=2) * 0.3
        add(f"coincident[{k}]", np.vstack([np.repeat(p[:, None], 4, 1), np.ones(4)]))
    for k in range(6):
        add(f"tiny_spread[{k}]", np.vstack([rng.normal(size=2)[:, None] * 0.5 + rng.normal(size=(2, 4)) * 1e-7,
                                            np.ones(4)]))
    for k in range(6):
        add(f"huge_spread[{k}]", np.vstack([rng.normal(size=(2, 4)) * rng.uniform(5, 200), np.ones(4)]))
    out = {"model": np.array(models), "iprts": np.array(iprts), "name": np.array(names)}
    st, Rs, ts, es = [], [], [], []
    for m, ip in zip(models, iprts):
        a, R, t, e = ref_case(m, ip)
        st.append(a)
        Rs.append(R)
        ts.append(t)
        es.append(e)
    out.update(status=np.array(st, np.int32), R=np.array(Rs), t=np.array(ts), errs=np.array(es))
    return out


def demo_case():
    md = [0.0685, 0.6383, 0.4558, 0.7411, -0.7219, 0.7081, 0.7061, 0.2887, -0.9521, -0.2553,
          0.4636, 0.0159, -0.1010, 0.2817, 0.6638, 0.1582, 0.3925, -0.7954, 0.6965, -0.7795]
    ipd = [-0.0168, 0.0377, 0.0277, 0.0373, -0.0824, 0.0386, 0.0317, 0.0360, -0.1015, -0.0080,
           0.0866, 0.1179, 0.1233, 0.1035, 0.0667, 0.1102, 0.0969, 0.1660, 0.0622, 0.1608]
    model = np.zeros((3, 10))
    ip = np.ones((3, 10))
    model[0], model[1] = md[:10], md[10:]
    ip[0], ip[1] = ipd[:10], ipd[10:]
    st, R, t, e = ref_case(model, ip)
    matlab_R = np.array([[0.85763, -0.31179, 0.40898], [0.16047, -0.59331, -0.78882], [0.48859, 0.74214, -0.45881]])
    matlab_t = np.array([-0.10825, 1.26601, 11.19855])
    return dict(model=model, iprts=ip, status=np.int32(st), R=R, t=t, errs=e, matlab_R=matlab_R, matlab_t=matlab_t)


def rpoly_cases():
    rng = np.random.default_rng(99)
    coefs = [np.poly([1.0, 2.0, 3.0, 4.0])]  # demo of the slot-4 quirk
    for _ in range(300):
        c = rng.normal(size=5) * 10.0 ** rng.integers(-3, 4, size=5)
        if c[0] == 0:
            c[0] = 1.0
        coefs.append(c)
    zr, zi, deg = [], [], []
    for c in coefs:
        d, r, i = O.rpoly(c, ref_impl=True)
        deg.append(d)
        zr.append(r)
        zi.append(i)
    return dict(coef=np.array(coefs), degree=np.array(deg, np.int32), zr=np.array(zr), zi=np.array(zi))


def grid1_case():
    from PIL import Image

    rgb = np.asarray(Image.open(REF_GRID1).convert("RGB"))
    bgr = np.ascontiguousarray(rgb[:, :, ::-1])
    h, w = bgr.shape[:2]
    K = np.array([450.0, 0, 453, 0, 450, 252, 0, 0, 1])
    D = np.zeros(4)
    white, red, green = synth.load_map()
    orc = O.Oracle(white, red, green, seed=1)
    dbg = orc.process(bgr, K, D)
    quads = np.array(dbg.quads, np.int32)[: dbg.n_quads]
    return dict(bgr=bgr, K=K, D=D, quads=quads, n_raw_quads=np.int32(dbg.n_raw_quads),
                reason=np.int32(dbg.reason), publish=np.int32(dbg.publish), n_hyps=np.int32(dbg.n_hyps),
                pub_error=np.float64(dbg.pub_error), position=np.array(dbg.position),
                rng_state_after=np.uint64(dbg.rng_state_after))


def main():
    if O.ref() is None:
        sys.exit("oracle/_ref/libref_rpoly.so missing: run `make ref` first")
    only = sys.argv[1:]  # e.g. `make_golden.py rpp_faults`: regenerate those fixtures only
    if only:
        for name in only:
            fn = {"rpp_faults": rpp_fault_cases}[name]
            np.savez_compressed(os.path.join(HERE, name + ".npz"), **fn())
            print(name, os.path.getsize(os.path.join(HERE, name + ".npz")))
        return
    np.savez_compressed(os.path.join(HERE, "rpp_golden.npz"), **rpp_cases())
    np.savez_compressed(os.path.join(HERE, "rpp_faults.npz"), **rpp_fault_cases())
    np.savez_compressed(os.path.join(HERE, "rpp_demo.npz"), **demo_case())
    np.savez_compressed(os.path.join(HERE, "rpoly_golden.npz"), **rpoly_cases())
    if os.path.exists(REF_GRID1):
        np.savez_compressed(os.path.join(HERE, "grid1.npz"), **grid1_case())
    for f in sorted(os.listdir(HERE)):
        print(f, os.path.getsize(os.path.join(HERE, f)))


if __name__ == "__main__":
    main()
