"""Probe: does the drop-in chain recycle its page-locked blocks? (GPU box)"""
import os, random, sys, time, types
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "stereo.vision_amd"), os.path.join(REPO, "tests")]
import numpy as np
import oracle
from svx import _abi, dropin
from test_prepass_cpu import carmask
f = types.SimpleNamespace(camera_focal_length_px=399.9745178222656, stereo_camera_baseline_m=0.2090607502,
                          image_centre_w=474.5, image_centre_h=262.0, carmask=carmask())
dropin.install(f, unpinned=True)
disp, bgr = oracle.synth_frame(0)
random.seed(0)
for it in range(6):
    t0 = time.perf_counter()
    points = f.projectDisparityTo3d(disp, 128, bgr)
    t1 = time.perf_counter()
    mp = f.projectDisparityTo3d(f.maskDisparity(disp), 128)
    _, abc = f.RANSAC(mp, 600)
    diffs = f.calculatePointErrors(abc, points)
    points = f.computePlanarThreshold(points, diffs, 0.05)
    hist = f.calculateColourHistogram(points)
    points = f.filterPointsByHistogram(points, hist, 10)
    pp = np.array(f.project3DPointsTo2DImagePoints(points), np.int32).reshape((-1, 1, 2))
    t2 = time.perf_counter()
    print(f"iter {it}: a1 {1e3 * (t1 - t0):.3f} ms, chain {1e3 * (t2 - t0):.3f} ms, pool allocs {_abi._pool.allocs}, "
          f"free {[(k, len(v)) for k, v in _abi._pool._free.items()]}", flush=True)
