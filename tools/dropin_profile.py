"""Per-call wall time of stereovision.py:84-113 through the installed drop-ins (one synthetic frame, step 2)."""
import os
import random
import sys
import time
import types

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "stereo.vision_amd"), os.path.join(ROOT, "tests")):
    sys.path.insert(0, p)
import oracle  # noqa: E402
from svx import dropin  # noqa: E402
from test_prepass_cpu import carmask  # noqa: E402

f = types.SimpleNamespace(camera_focal_length_px=399.9745178222656, stereo_camera_baseline_m=0.2090607502,
                          image_centre_w=474.5, image_centre_h=262.0, carmask=carmask())
dropin.install(f)
disp, bgr = oracle.synth_frame(0)
T = {}


def t(name, fn, *a):
    t0 = time.perf_counter()
    r = fn(*a)
    T[name] = T.get(name, 0.0) + (time.perf_counter() - t0) * 1e3
    return r


random.seed(0)
for rep in range(6):
    if rep == 1:
        T.clear()
    points = t("a1 projectDisparityTo3d(rgb)", f.projectDisparityTo3d, disp, 128, bgr)
    md = t("maskDisparity", f.maskDisparity, disp)
    mp = t("a1 projectDisparityTo3d(mask)", f.projectDisparityTo3d, md, 128)
    _, abc = t("RANSAC(600)", f.RANSAC, mp, 600)
    diffs = t("a2 calculatePointErrors", f.calculatePointErrors, abc, points)
    points = t("a3 computePlanarThreshold", f.computePlanarThreshold, points, diffs, 0.05)
    hist = t("a5 calculateColourHistogram", f.calculateColourHistogram, points)
    points = t("a6 filterPointsByHistogram", f.filterPointsByHistogram, points, hist, 10)
    pp = t("a7 project3DPointsTo2DImagePoints", f.project3DPointsTo2DImagePoints, points)
    t("a8 int32 cast", lambda: np.array(pp, np.int32).reshape((-1, 1, 2)))
for k, v in T.items():
    print(f"{k:40s} {v / 5:8.2f} ms")
print(f"{'total':40s} {sum(T.values()) / 5:8.2f} ms")
