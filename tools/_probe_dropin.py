"""Scratch probe: where the drop-in projection's host time goes (GPU box)."""
import ctypes, os, sys, time
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "stereo.vision_amd")]
import numpy as np
import oracle
from svx import dropin, _abi
import types
f = types.SimpleNamespace(camera_focal_length_px=399.9745178222656, stereo_camera_baseline_m=0.2090607502,
                          image_centre_w=474.5, image_centre_h=262.0)
dropin.install(f)
disp, bgr = oracle.synth_frame(0)
def t(name, fn, reps=20):
    fn()
    t0 = time.perf_counter()
    for _ in range(reps): fn()
    print(f"{name:40s} {(time.perf_counter() - t0) / reps * 1e3:8.3f} ms", flush=True)
t("projectDisparityTo3d(rgb)", lambda: f.projectDisparityTo3d(disp, 128, bgr))
t("project_frame(rgb)", lambda: dropin.project_frame(disp, bgr))
t("project_frame(no rgb)", lambda: dropin.project_frame(disp, None))
h, w = disp.shape
cap = 543 * 512
xyz = np.empty((cap, 3)); rgb = np.empty((cap, 3), np.uint8); n = ctypes.c_int64(0)
cam = dropin._camera()
t("sv_project_frame warm outputs (rgb)", lambda: _abi.call("sv_project_frame", _abi.ptr(disp), h, w, w, _abi.ptr(bgr), 3 * w, 2, ctypes.byref(cam), _abi.ptr(xyz), _abi.ptr(rgb), cap, ctypes.byref(n)))
t("sv_project_frame warm outputs (no rgb)", lambda: _abi.call("sv_project_frame", _abi.ptr(disp), h, w, w, None, 0, 2, ctypes.byref(cam), _abi.ptr(xyz), None, cap, ctypes.byref(n)))
t("np.empty 3.3MB + touch", lambda: np.empty((cap, 3)).fill(0))
pts = f.projectDisparityTo3d(disp, 128, bgr)
t("project3DPointsTo2DImagePoints", lambda: f.project3DPointsTo2DImagePoints(pts))
