"""ORACLE (test infrastructure only): the nested-loop CPU port.

A scalar, interpreter-level restatement of the reference hot path with the
same numpy-scalar semantics (fp64 XYZ, uint8 colour channels, numpy rounding,
colorsys hue). It is the CPU baseline timed by ``bench.py`` on the GPU box
(the reference itself cannot travel there) and a second, independent checker
for small cases. Its parity with the reference is pinned by tests/golden/.

Reference lines restated (thien/stereo.vision):
  project          functions.py:178-198  (grid step generalised; ref = 2)
  backproject      functions.py:201-209
  hue_key          functions.py:73-78 (+ colorsys.rgb_to_hsv)
  point_errors     functions.py:300-312
  plane_keep       functions.py:314-323
  colour_hist      functions.py:215-226
  hist_keep        functions.py:228-230
  chain            stereovision.py:84,97-113
"""
import colorsys
import math

import numpy as np

from . import CH, CW, F_PX, BASELINE_M


def project(disp, bgr=None, step=2, f=F_PX, B=BASELINE_M, cw=CW, ch=CH):
    """Rows [X, Y, Z(, R, G, B)] in raster order for every grid pixel with d > 0."""
    rows = []
    fb = f * B
    h, w = disp.shape[:2]
    want_rgb = bgr is not None and len(bgr) > 0
    for y in range(0, h - 1, step):
        line = disp[y]
        for x in range(0, w - 1, step):
            d = line[x]                      # numpy uint8 scalar
            if not d > 0:
                continue
            z = fb / d                       # python float / np.uint8 -> np.float64
            px = ((x - cw) * z) / f
            py = ((y - ch) * z) / f
            if want_rgb:
                c = bgr[y, x]
                rows.append([px, py, z, c[2], c[1], c[0]])
            else:
                rows.append([px, py, z])
    return rows


def backproject(rows, f=F_PX, cw=CW, ch=CH):
    out = []
    for r in rows:
        z = r[2]
        out.append([((r[0] * f) / z) + cw, ((r[1] * f) / z) + ch])
    return out


def hue_key(r, g, b):
    """str(round(hue, 3)) of colorsys HSV on numpy-scalar channels."""
    return str(round(colorsys.rgb_to_hsv(r, g, b)[0], 3))


def point_errors(abc, rows):
    pts = np.array([[r[0], r[1], r[2]] for r in rows])
    a, b, c = (float(v) for v in np.asarray(abc).reshape(3))
    nrm = math.sqrt(a * a + b * b + c * c)
    return abs((np.dot(pts, abc) - 1) / nrm)


def plane_keep(rows, dist, thr):
    return [r for r, e in zip(rows, dist) if e < thr]


def colour_hist(rows):
    hist = {}
    for r in rows:
        k = hue_key(r[3], r[4], r[5])
        hist[k] = hist.get(k, 0) + 1
    return hist


def hist_keep(rows, hist, thr):
    return [r for r in rows if hist[hue_key(r[3], r[4], r[5])] > thr]


def chain(disp, bgr, abc, step=2, point_thr=0.05, hist_thr=10):
    """Returns (rows, kept, kept2, plane_points int32 (N2,1,2), hist dict)."""
    abc = np.asarray(abc, np.float64).reshape(3, 1)
    rows = project(disp, bgr, step)
    dist = point_errors(abc, rows) if rows else np.zeros((0, 1))
    kept = plane_keep(rows, dist, point_thr)
    hist = colour_hist(kept)
    kept2 = hist_keep(kept, hist, hist_thr)
    pp = np.array(backproject(kept2), np.int32).reshape((-1, 1, 2))
    return rows, kept, kept2, pp, hist


def key_to_bin(key):
    return int(round(float(key) * 1000))
