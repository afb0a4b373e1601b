"""ORACLE — test infrastructure only: the disparity stage upstream of the hot path.

Python side of ``oracle/sgbm_oracle.c`` (functions.py:61-128):
``gamma_table`` / ``gamma_change`` restate functions.py:61-67 with the same
numpy expression; ``grey_equalize`` = cv2.cvtColor(BGR2GRAY) + equalizeHist
(functions.py:89-97); ``sgbm`` = StereoSGBM(0, 128, 21).compute;
``sgbm_raw`` = computeDisparitySGBM alone, ``median3`` = the medianBlur(disp, disp, 3)
StereoSGBM::compute runs after it; ``filter_speckles``; ``disparity`` =
functions.py:104-128 end to end.
``synth_pair`` is the numpy twin of the device's synthetic rectified pair.

PARITY UNPINNED for the cv2 calls (cv2 is absent here; see sgbm_oracle.c).
"""
import ctypes

import numpy as np

from . import _p, c_lib
from .synth import mix64 as svo_mix64_np

# StereoSGBM_create(0, max_disparity, 21) with OpenCV's defaults for the rest
# (functions.py:26): P1 = P2 = 0 -> 2 / 5, disp12MaxDiff 0 -> 1, preFilterCap
# 0 -> 15, uniquenessRatio 0, speckleWindowSize 0, mode MODE_SGBM.
REFERENCE_PARAMS = dict(min_disp=0, num_disp=128, block=21, P1=0, P2=0, disp12_max_diff=0,
                        prefilter_cap=0, uniqueness=0)


class SgbmParams(ctypes.Structure):
    _fields_ = [(k, ctypes.c_int) for k in ("min_disp", "num_disp", "block", "P1", "P2", "disp12_max_diff",
                                            "prefilter_cap", "uniqueness")]


def params(**kw):
    p = dict(REFERENCE_PARAMS)
    p.update(kw)
    return SgbmParams(**p)


def _lib():
    lib = c_lib()
    if not getattr(lib, "_sgbm_bound", False):
        P, ci = ctypes.c_void_p, ctypes.c_int
        lib.svo_grey_equalize.argtypes = [P, ci, ci, P]
        lib.svo_grey_equalize.restype = None
        lib.svo_sgbm.argtypes = [P, P, ci, ci, P, P]
        lib.svo_sgbm.restype = ci
        lib.svo_sgbm_compute.argtypes = [P, P, ci, ci, P, P]
        lib.svo_sgbm_compute.restype = ci
        lib.svo_median3_s16.argtypes = [P, ci, ci, P]
        lib.svo_median3_s16.restype = None
        lib.svo_filter_speckles.argtypes = [P, ci, ci, ci, ci, ci]
        lib.svo_filter_speckles.restype = ci
        lib.svo_disparity_scale.argtypes = [P, ci, ci, ci, ci, P]
        lib.svo_disparity_scale.restype = None
        lib._sgbm_bound = True
    return lib


def gamma_table(gamma=1.4):
    """functions.py:61-67, the same numpy expression (astype('uint8') truncates)."""
    inv = 1.0 / gamma
    return np.array([((i / 255.0) ** inv) * 255 for i in np.arange(0, 256)]).astype("uint8")


def gamma_change(img, gamma=1.4):
    """cv2.LUT(image, table) for a uint8 image and a 256-entry uint8 table."""
    return gamma_table(gamma)[img]


def grey_equalize(bgr):
    bgr = np.ascontiguousarray(bgr, np.uint8)
    H, W = bgr.shape[:2]
    out = np.empty((H, W), np.uint8)
    _lib().svo_grey_equalize(_p(bgr), H, W, _p(out))
    return out


def _sgbm_call(fn, left, right, kw):
    left = np.ascontiguousarray(left, np.uint8)
    right = np.ascontiguousarray(right, np.uint8)
    if left.shape != right.shape or left.ndim != 2:
        raise ValueError(f"left {left.shape} and right {right.shape} must be equal 2-D shapes")
    H, W = left.shape
    out = np.empty((H, W), np.int16)
    prm = params(**kw)
    rc = fn(_p(left), _p(right), H, W, ctypes.byref(prm), _p(out))
    if rc:
        raise ValueError("svo_sgbm: unsupported geometry (rc=%d)" % rc)
    return out


def sgbm(left, right, **kw):
    """StereoSGBM.compute(left, right): (H, W) int16 disparity x16
    (computeDisparitySGBM, then medianBlur 3 as OpenCV's compute does)."""
    return _sgbm_call(_lib().svo_sgbm_compute, left, right, kw)


def sgbm_raw(left, right, **kw):
    """computeDisparitySGBM alone (before compute's medianBlur)."""
    return _sgbm_call(_lib().svo_sgbm, left, right, kw)


def median3(d16):
    """cv2.medianBlur(d16, 3) on int16: exact 3 x 3 median, replicated border."""
    d16 = np.ascontiguousarray(d16, np.int16)
    H, W = d16.shape
    out = np.empty_like(d16)
    _lib().svo_median3_s16(_p(d16), H, W, _p(out))
    return out


def filter_speckles(d16, new_val=0, max_size=4000, max_diff=123):
    out = np.ascontiguousarray(d16, np.int16).copy()
    H, W = out.shape
    _lib().svo_filter_speckles(_p(out), H, W, int(new_val), int(max_size), int(max_diff))
    return out


def scale(d16, max_disparity=128, crop=False):
    d16 = np.ascontiguousarray(d16, np.int16)
    H, W = d16.shape
    rows, cols = (min(390, H), max(W - 135, 0)) if crop else (H, W)
    out = np.empty((rows, cols), np.uint8)
    _lib().svo_disparity_scale(_p(d16), H, W, int(max_disparity), int(bool(crop)), _p(out))
    return out


def disparity(grey_l, grey_r, max_disparity=128, crop=False, with_raw=False, **kw):
    """functions.py:104-128: SGBM -> filterSpeckles(0, 4000, max_disparity - 5)
    -> TOZERO -> /16 -> u8 -> optional crop -> x(256 / max_disparity) -> u8."""
    raw = sgbm(grey_l, grey_r, num_disp=max_disparity, **kw)
    filt = filter_speckles(raw, 0, 4000, max_disparity - 5)
    out = scale(filt, max_disparity, crop)
    return (out, raw, filt) if with_raw else out


# ---------------------------------------------------------------------------
# Synthetic rectified pair (numpy twin of sgbm.hip synth_pair_kernel).
# Texture T(frame, y, u) from the counter hash; the true disparity of row y is
# the synthetic road's, halved to SGBM units: D(y) = clamp(floor(3(y - 200) / 10), 0, 127).
# left(y, x) = T(y, x), right(y, x) = T(y, x + D(y)), so left x matches right x - D(y).
# ---------------------------------------------------------------------------
PAIR_SALT = 0x57E2E0000000000


def pair_true_disparity(H):
    y = np.arange(H, dtype=np.int64)
    return np.clip(np.floor_divide(3 * (y - 200), 10), 0, 127)


def pair_texture(frame_id, H, W_ext):
    y = np.arange(H, dtype=np.uint64)[:, None]
    u = np.arange(W_ext, dtype=np.uint64)[None, :]
    idx = (np.uint64(frame_id) * np.uint64(H) + y) * np.uint64(4096) + u
    h = svo_mix64_np(idx + np.uint64(PAIR_SALT))
    return (np.uint64(48) + (h & np.uint64(0x9F))).astype(np.uint8)


def synth_pair(frame_id, H=544, W=1024):
    T = pair_texture(frame_id, H, W + 128)
    D = pair_true_disparity(H)
    left = np.ascontiguousarray(T[:, :W])
    xs = np.arange(W)[None, :] + D[:, None]
    right = np.ascontiguousarray(np.take_along_axis(T, xs, axis=1))
    return left, right
