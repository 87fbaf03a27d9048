"""cv::Canny's hysteresis as a stage of its own.

The reference's hysteresis is OpenCV's stack walk (QuadDetection.h:212 and
HypothesisEvaluation.h:327 call cv::Canny; the walk is restated in
oracle/o_imgproc.cpp hysteresis_walk). The library runs it as a bit-parallel
reconstruction (k_hyst_rec, one block per frame up to 720 rows) or as a run
CCL (k_hyst_band / _seam / _mark / _fix: taller frames, MANTIS_HYST_REC=0).

CPU: the oracle's walk equals the 8-connected components of the candidates
that hold a strong pixel (scipy.ndimage.label), the set the reconstruction
computes. GPU: both device paths against the oracle's walk, bit for bit, on
class planes built to stress the reconstruction: serpentines whose reach
changes direction at every column (one sweep per turn), spirals, weak lines
through every band seam seeded from either end, random planes of every
density, frames ending mid-band and mid-word, and the empty / full cases.
"""
import os

import numpy as np
import pytest

import _oracle as O


def _components_ref(cls):
    from scipy import ndimage

    cand = cls > 0
    lab, n = ndimage.label(cand, structure=np.ones((3, 3), bool))
    keep = np.zeros(n + 1, bool)
    keep[np.unique(lab[cls == 2])] = True
    keep[0] = False
    return np.where(keep[lab], 255, 0).astype(np.uint8)


def _serpentine(h, w, gap=2, strong_at="top"):
    """vertical candidate lines every `gap` columns joined alternately at the
    bottom and the top: the reach turns at every line"""
    cls = np.zeros((h, w), np.uint8)
    xs = list(range(0, w, gap))
    for k, x in enumerate(xs):
        cls[:, x] = 1
        if k + 1 < len(xs):
            y = h - 1 if k % 2 == 0 else 0
            cls[y, x:xs[k + 1] + 1] = 1
    if strong_at == "top":
        cls[0, 0] = 2
    else:
        cls[h - 1 if (len(xs) - 1) % 2 == 0 else 0, xs[-1]] = 2
    return cls


def _spiral(h, w):
    cls = np.zeros((h, w), np.uint8)
    top, left, bottom, right = 0, 0, h - 1, w - 1
    while top <= bottom and left <= right:
        cls[top, left:right + 1] = 1
        cls[top:bottom + 1, right] = 1
        if top + 2 <= bottom:
            cls[bottom, left:right + 1] = 1
        if left + 2 <= right:
            cls[top + 2:bottom + 1, left] = 1
        top, left, bottom, right = top + 2, left + 2, bottom - 2, right - 2
    # the innermost end: strong
    ys, xs = np.nonzero(cls)
    c = np.argmin(np.abs(ys - h / 2) + np.abs(xs - w / 2))
    cls[ys[c], xs[c]] = 2
    return cls


def _cases():
    rng = np.random.default_rng(2024)
    out = []
    for (w, h, dens, p_strong) in [(1280, 720, 0.35, 0.002), (1280, 720, 0.55, 0.0005), (907, 505, 0.45, 0.001),
                                   (33, 7, 0.6, 0.05), (130, 91, 0.5, 0.01), (2016, 700, 0.4, 0.001),
                                   (1920, 1080, 0.4, 0.001), (64, 720, 0.7, 0.0002)]:
        cand = rng.random((h, w)) < dens
        strong = cand & (rng.random((h, w)) < p_strong)
        out.append((f"random{w}x{h}d{dens}", np.where(strong, 2, np.where(cand, 1, 0)).astype(np.uint8)))
    out.append(("serpentine_top", _serpentine(720, 1280, 2, "top")))
    out.append(("serpentine_end", _serpentine(720, 1280, 3, "end")))
    out.append(("serpentine_short", _serpentine(97, 301, 2, "top")))
    out.append(("spiral", _spiral(720, 1280)))
    out.append(("spiral_odd", _spiral(333, 517)))
    # weak vertical / diagonal lines through every band seam, strong only at one end
    cls = np.zeros((720, 1280), np.uint8)
    for x in range(5, 1280, 37):
        cls[:, x] = 1
        cls[0 if (x // 37) % 2 else 719, x] = 2
    for k in range(0, 1200, 150):  # diagonals crossing seams between rows
        for y in range(720):
            x = k + y // 2
            if x < 1280:
                cls[y, x] = max(cls[y, x], 1)
        cls[719, min(1279, k + 359)] = 2
    out.append(("seam_lines", cls))
    # lines on the band boundary rows (44 / 45, 89 / 90 ...) and words' edge columns
    cls = np.zeros((720, 1280), np.uint8)
    for y in range(44, 720, 45):
        cls[y, 31:1249] = 1
        cls[y + 1 if y + 1 < 720 else y, 32:1250:2] = 1
    cls[44, 31] = 2
    out.append(("band_rows", cls))
    out.append(("empty", np.zeros((720, 1280), np.uint8)))
    out.append(("all_weak", np.ones((720, 1280), np.uint8)))
    full = np.ones((100, 200), np.uint8)
    full[99, 199] = 2
    out.append(("all_one_strong", full))
    return out


def test_oracle_walk_equals_strong_components():
    for name, cls in _cases():
        if cls.size > 1_000_000 and name.startswith("random"):
            continue  # the scipy reference is fine; keep the CPU suite short
        got = O.hysteresis(cls)
        ref = _components_ref(cls)
        assert np.array_equal(got, ref), f"{name}: {np.count_nonzero(got != ref)} px differ"


@pytest.mark.gpu
@pytest.mark.parametrize("rec", ["1", "0"])
def test_hysteresis_device_paths_match_oracle(rec):
    import mantis_amd as M

    saved = os.environ.get("MANTIS_HYST_REC")
    os.environ["MANTIS_HYST_REC"] = rec
    try:
        m = M.Mantis(max_cams=1, max_width=2016, max_height=1080)
    finally:
        if saved is None:
            os.environ.pop("MANTIS_HYST_REC")
        else:
            os.environ["MANTIS_HYST_REC"] = saved
    try:
        for name, cls in _cases():
            got = m.hysteresis(cls)
            ref = O.hysteresis(cls)
            bad = np.argwhere(got != ref)
            assert len(bad) == 0, f"{name} (MANTIS_HYST_REC={rec}): {len(bad)} px differ, first {bad[:8].tolist()}"
    finally:
        m.close()


@pytest.mark.gpu
def test_ccl_epoch_wrap_stays_bit_exact():
    """The run CCL marks strong seam components with a per-call epoch byte and
    clears its flag plane only when the epoch wraps (255 -> 4): start the epoch
    at 252 (MANTIS_HYST_EPOCH0) and run the CCL path across the wrap on frames
    whose components reach band seams, each call bit-exact against the oracle
    (the wrap was never reached by a test)."""
    import mantis_amd as M
    from mantis_amd import synth

    env = {"MANTIS_HYST_REC": "0", "MANTIS_HYST_EPOCH0": "252"}
    saved = {k: os.environ.get(k) for k in env}
    os.environ.update(env)
    try:
        m = M.Mantis(max_cams=1, max_width=1280, max_height=720)
    finally:
        for k, v in saved.items():
            if v is None:
                os.environ.pop(k)
            else:
                os.environ[k] = v
    try:
        rng = np.random.default_rng(99)
        K, D = synth.intrinsics()
        for call in range(8):  # epochs 253, 254, 255, 4 (plane cleared), 5, ...
            base = rng.integers(0, 256, (720 // 6 + 2, 1280 // 6 + 2, 3)).astype(np.float64)
            img = np.repeat(np.repeat(base, 6, 0), 6, 1)[:720, :1280]
            img = np.clip(img + rng.normal(0, 20, img.shape), 0, 255).astype(np.uint8)
            got = m.canny(M.make_image(img, K, D))
            ref = O.canny(img)
            assert np.array_equal(got, ref), f"call {call}: {np.count_nonzero(got != ref)} px differ"
            cls = _cases()[call % 4][1]
            assert np.array_equal(m.hysteresis(cls), O.hysteresis(cls)), f"call {call}: hysteresis stage differs"
    finally:
        m.close()
