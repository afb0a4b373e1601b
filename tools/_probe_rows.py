"""Probe: the drop-in projection's rows into pageable vs pooled page-locked memory (GPU box): the device call, the
CPU reading the result, and the pool's reuse."""
import ctypes, os, sys, time
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "stereo.vision_amd")]
import numpy as np
import oracle
from svx import _abi, dropin
disp, bgr = oracle.synth_frame(0)
h, w = disp.shape
cap = 543 * 512
cam = dropin._camera()
n = ctypes.c_int64(0)
def t(name, fn, reps=20):
    fn()
    t0 = time.perf_counter()
    for _ in range(reps): fn()
    print(f"{name:52s} {(time.perf_counter() - t0) / reps * 1e3:8.3f} ms", flush=True)
page = np.empty((cap, 6), np.float64)
pin = _abi.pinned_empty((cap, 6), np.float64)
def rows_into(a):
    _abi.call("sv_project_rows", _abi.ptr(disp), h, w, w, _abi.ptr(bgr), 3 * w, 2, ctypes.byref(cam), _abi.ptr(a),
              6, cap, ctypes.byref(n))
t("sv_project_rows -> pageable", lambda: rows_into(page))
t("sv_project_rows -> pinned", lambda: rows_into(pin))
t("CPU sum over pageable rows", lambda: page[: n.value].sum())
t("CPU sum over pinned rows", lambda: pin[: n.value].sum())
t("pinned_empty (pool reuse)", lambda: _abi.pinned_empty((cap, 6), np.float64))
t("np.empty + touch", lambda: np.empty((cap, 6)).fill(0))
t("dropin.project_rows", lambda: dropin.project_rows(disp, bgr))
t("dropin.projectDisparityTo3d", lambda: dropin.projectDisparityTo3d(disp, 128, bgr))
xyz = np.empty((cap, 3)); rgb = np.empty((cap, 3), np.uint8)
t("sv_project_frame (pageable xyz + rgb)", lambda: _abi.call("sv_project_frame", _abi.ptr(disp), h, w, w, _abi.ptr(bgr),
  3 * w, 2, ctypes.byref(cam), _abi.ptr(xyz), _abi.ptr(rgb), cap, ctypes.byref(n)))
