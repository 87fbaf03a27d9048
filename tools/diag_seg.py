"""Diagnostic of the segmented border walks (GPU box): the throughput walker
(MANTIS_TRACE_LDS_FRAMES=0) on blob-noise frames at several checkpoint
spacings (MANTIS_SEG_M), frame counters and the oracle's contour totals."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests")]
import _oracle as O
import mantis_amd as M
from mantis_amd import synth

K, D = synth.intrinsics()
rng = np.random.default_rng(123)
imgs = []
for (w, h, cell) in [(333, 97, 2), (1000, 611, 6), (640, 480, 3), (1280, 720, 6)]:
    base = (rng.random((h // cell + 2, w // cell + 2)) > 0.5).astype(np.float64) * 200 + 20
    img = np.repeat(np.repeat(base, cell, 0), cell, 1)[:h, :w]
    imgs.append(np.repeat(img[:, :, None], 3, 2).astype(np.uint8))
os.environ["MANTIS_TRACE_LDS_FRAMES"] = "0"
for segm in sys.argv[1:] or ["0", "32"]:
    os.environ["MANTIS_SEG_M"] = segm
    mt = M.Mantis(max_cams=2, max_width=1280, max_height=720)
    for img in imgs:
        try:
            mt.detect_quads(M.make_image(img, K, D))
            err = ""
        except M.MantisError as e:
            err = str(e)[:60]
        c = mt.frame_counters(0)
        cs, holes = O.find_contours(O.detector_binary(O.canny(img)), 2)
        print(f"M={segm} {img.shape[1]}x{img.shape[0]}: borders {c[0]}/{len(cs)} points {c[1]}/{sum(len(x) for x in cs)} "
              f"overflow {c[8]} runs {c[9]} chunks {c[19]} seg_nc {c[22]} seg_m {c[23]} steps {c[20]} {err}")
    mt.close()
