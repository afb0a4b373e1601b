"""ORACLE (test infrastructure only): the reference's hot-path loops as written.

``oracle/cpu_loop.py`` is a port with the loop invariants hoisted (f*B once, the
row indexed once, the colour indexed once per point). This module is the
literal form the reference actually runs, so that bench.py's config-1 CPU
baseline times the reference's own interpreter work, not a tidier loop:

  project            functions.py:178-198  disparity[y,x] read twice per valid
                                           point, f*B evaluated per point, the
                                           module globals image_centre_w / _h
                                           looked up per point, len(rgb)
                                           tested per point, rgb[y,x,c] three
                                           times
  backproject        functions.py:201-209  index loop, points[i1][k] per use,
                                           module-global focal length per use
  hue                functions.py:69-78    getPointColour + BGRtoHSVHue
  colour_hist        functions.py:215-226  list of keys, then the dict loop
  hist_keep          functions.py:228-230  comprehension, key recomputed
  point_errors       functions.py:300-312  list rebuild with append, math.sqrt
                                           on (1,)-arrays, BLAS dot
  plane_keep         functions.py:314-323  index loop with append
  ransac             functions.py:240-298  random.sample on the row list, the
                                           sampled rows re-wrapped by np.array /
                                           np.dot per trial, exceptions swallowed
  chain              stereovision.py:84,97-113

Same numpy-scalar semantics as the reference (np.uint8 disparity and colours,
np.float64 XYZ): its outputs are pinned to tests/golden/ like cpu_loop's
(tests/test_oracle_golden.py). Never imported by the product.
"""
import colorsys
import math
import random

import numpy as np

from . import CH, CW, F_PX, BASELINE_M

# module-level constants looked up as globals inside the loops, as functions.py:15-22 are
camera_focal_length_px = F_PX
stereo_camera_baseline_m = BASELINE_M
image_centre_w = CW
image_centre_h = CH


def project(disparity, max_disparity, rgb=[]):  # noqa: B006 (the reference's signature)
    points = []
    f = camera_focal_length_px
    B = stereo_camera_baseline_m
    height, width = disparity.shape[:2]
    for y in range(0, height - 1, 2):
        for x in range(0, width - 1, 2):
            if disparity[y, x] > 0:
                Z = (f * B) / disparity[y, x]
                X = ((x - image_centre_w) * Z) / f
                Y = ((y - image_centre_h) * Z) / f
                if len(rgb) > 0:
                    points.append([X, Y, Z, rgb[y, x, 2], rgb[y, x, 1], rgb[y, x, 0]])
                else:
                    points.append([X, Y, Z])
    return points


def backproject(points):
    pts = []
    for i1 in range(len(points)):
        Z = points[i1][2]
        x = ((points[i1][0] * camera_focal_length_px) / Z) + image_centre_w
        y = ((points[i1][1] * camera_focal_length_px) / Z) + image_centre_h
        pts.append([x, y])
    return pts


def point_colour(point):
    return (point[3], point[4], point[5])


def hue(rgb):
    r, g, b = rgb
    h = round(colorsys.rgb_to_hsv(r, g, b)[0], 3)
    return str(h)


def colour_hist(points):
    colours = [hue((pt[3], pt[4], pt[5])) for pt in points]
    histogram = {}
    for i in colours:
        if i not in histogram:
            histogram[i] = 1
        else:
            histogram[i] += 1
    return histogram


def hist_keep(points, histogram, threshold=100):
    return [x for x in points if histogram[hue(point_colour(x))] > threshold]


def point_errors(abc, points):
    the_list = []
    for i in points:
        the_list.append([i[0], i[1], i[2]])
    pts = np.array(the_list)
    d = math.sqrt(abc[0] * abc[0] + abc[1] * abc[1] + abc[2] * abc[2])
    return abs((np.dot(pts, abc) - 1) / d)


def plane_keep(points, differences, threshold=0.01):
    new_points = []
    for i in range(len(points)):
        if differences[i] < threshold:
            new_points.append(points[i])
    return new_points


def non_collinear(points):
    check = np.array([0, 0, 0])
    c0, c1, c2 = check[0] == 0, check[1] == 0, check[2] == 0
    P1 = P2 = P3 = None
    while c0 and c1 and c2:
        P1 = np.array([x[:3] for x in random.sample(points, 1)])[0]
        P2 = np.array([x[:3] for x in random.sample(points, 1)])[0]
        P3 = np.array([x[:3] for x in random.sample(points, 1)])[0]
        check = np.cross(P1 - P2, P2 - P3)
        c0, c1, c2 = check[0] == 0, check[1] == 0, check[2] == 0
    return (P1, P2, P3)


def plane_fit(sample, points):
    P1, P2, P3 = non_collinear(points)
    abc = np.dot(np.linalg.inv(np.array([P1, P2, P3])), np.ones([3, 1]))
    d = math.sqrt(abc[0] * abc[0] + abc[1] * abc[1] + abc[2] * abc[2])
    if len(sample[0]) > 3:
        sample = [[item[0], item[1], item[2]] for item in sample]
    dist = abs((np.dot(sample, abc) - 1) / d)
    return abc, abc, dist


def ransac(points, trials):
    """(normal, coefficients) of the best plane, or (None, None); draws from the global `random`."""
    best = (None, None)
    best_err = float("inf")
    for _ in range(trials):
        try:
            T = random.sample(points, 600)
            coeffs, normal, dist = plane_fit(T, points)
            err = np.mean(dist)
            if err < best_err:
                best = (normal, coeffs)
                best_err = err
        except Exception:   # the reference swallows singular systems and short point lists alike
            pass
    return best


def chain(disp, bgr, abc, point_thr=0.05, hist_thr=10):
    """stereovision.py:84,97-113 for one frame at the reference's step 2:
    (points, kept, kept2, planePoints int32 (N2,1,2), hist dict)."""
    abc = np.asarray(abc, np.float64).reshape(3, 1)
    points = project(disp, 128, bgr)
    diffs = point_errors(abc, points)
    kept = plane_keep(points, diffs, point_thr)
    hist = colour_hist(kept)
    kept2 = hist_keep(kept, hist, hist_thr)
    pp = np.array(backproject(kept2), np.int32).reshape((-1, 1, 2))
    return points, kept, kept2, pp, hist
