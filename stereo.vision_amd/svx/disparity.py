"""Drop-ins for the disparity stage upstream of the hot path.

``performStereoVision`` (stereovision.py:40-62) runs, per stereo pair::

    imgL, imgR = f.preProcessImages(imgL, imgR)          functions.py:81-87 (gammaChange :61-67)
    grayL, grayR = f.greyscale(imgL, imgR)               functions.py:89-97
    disparity = f.disparity(grayL, grayR, 128, crop)     functions.py:104-128

All three are OpenCV calls in the reference (cv2.LUT, cvtColor + equalizeHist,
StereoSGBM + filterSpeckles + threshold). Here each is one device call
(kernels/sgbm.hip through include/svx.h): ``gammaChange`` builds the table
with the reference's own numpy expression and applies it on the GPU;
``greyscale`` is cvtColor(BGR2GRAY) + equalizeHist on the GPU; ``disparity``
is the whole SGBM stage on the GPU, with the parameters of the installed
module's ``stereoProcessor`` when it exposes OpenCV's getters, else the
reference's (0, 128, 21).

Same argument meaning, return types and shapes as the reference; failures
raise ``RuntimeError`` (``SvxError``), which stereovision.py:52-62 catches
like a cv2.error ("Cannot compute the disparity.").
"""
import ctypes

import numpy as np

from . import _abi

# functions.py:26 StereoSGBM_create(0, max_disparity=128, 21): other fields 0
REFERENCE_SGBM = dict(min_disp=0, num_disp=128, block=21, P1=0, P2=0, disp12_max_diff=0, prefilter_cap=0,
                      uniqueness=0)


class SgbmParams(ctypes.Structure):
    _fields_ = [(k, ctypes.c_int) for k in ("min_disp", "num_disp", "block", "P1", "P2", "disp12_max_diff",
                                            "prefilter_cap", "uniqueness")]


def sgbm_params(**kw):
    p = dict(REFERENCE_SGBM)
    unknown = set(kw) - set(p)
    if unknown:
        raise TypeError(f"unknown SGBM parameters {sorted(unknown)}")
    p.update(kw)
    return SgbmParams(**{k: int(v) for k, v in p.items()})


def _processor_params():
    """The installed module's stereoProcessor settings (cv2 getters), if any."""
    from . import dropin
    sp = getattr(dropin._module, "stereoProcessor", None) if dropin._module is not None else None
    if sp is None or not hasattr(sp, "getNumDisparities"):
        return sgbm_params()
    if sp.getSpeckleWindowSize() > 0 or sp.getMode() != 0:
        raise NotImplementedError("svx SGBM implements MODE_SGBM without the internal speckle window "
                                  "(the reference's configuration, functions.py:26)")
    return sgbm_params(min_disp=sp.getMinDisparity(), num_disp=sp.getNumDisparities(), block=sp.getBlockSize(),
                       P1=sp.getP1(), P2=sp.getP2(), disp12_max_diff=sp.getDisp12MaxDiff(),
                       prefilter_cap=sp.getPreFilterCap(), uniqueness=sp.getUniquenessRatio())


def _u8(a, what, ndim=None):
    arr = np.asarray(a)
    if arr.dtype != np.uint8:
        raise TypeError(f"{what} must be uint8, got {arr.dtype}")
    if ndim is not None and arr.ndim != ndim:
        raise ValueError(f"{what} must have {ndim} dimensions, got shape {arr.shape}")
    return np.ascontiguousarray(arr)


# ---------------------------------------------------------------------------
# functions.py:61-97
# ---------------------------------------------------------------------------
def gamma_table(gamma=1.0):
    """The table of functions.py:61-67 (the reference's numpy expression)."""
    inv = 1.0 / gamma
    return np.array([((i / 255.0) ** inv) * 255 for i in np.arange(0, 256)]).astype("uint8")


def apply_lut(image, table):
    """cv2.LUT(image, table) for uint8 images and a 256-entry uint8 table, on the GPU."""
    img = _u8(image, "image")
    lut = _u8(np.asarray(table).reshape(-1), "table")
    if lut.size != 256:
        raise ValueError("the table must have 256 entries")
    out = np.empty_like(img)
    _abi.call("sv_lut_u8", _abi.ptr(img), img.size, _abi.ptr(lut), _abi.ptr(out))
    return out


def gammaChange(image, gamma=1.0):  # noqa: N802
    """functions.py:61-67 (cv2.LUT on the GPU)."""
    return apply_lut(image, gamma_table(gamma))


def preProcessImages(imgL, imgR):  # noqa: N802
    """functions.py:81-87: gamma 1.4 on both images."""
    return gammaChange(imgL, 1.4), gammaChange(imgR, 1.4)


def grey_equalize(image):
    """cv2.equalizeHist(cv2.cvtColor(image, cv2.COLOR_BGR2GRAY)) on the GPU."""
    img = _u8(image, "image", 3)
    if img.shape[2] != 3:
        raise ValueError(f"expected a BGR image, got shape {img.shape}")
    H, W = img.shape[:2]
    out = np.empty((H, W), np.uint8)
    _abi.call("sv_grey_equalize", _abi.ptr(img), H, W, _abi.ptr(out))
    return out


def greyscale(imgL, imgR):  # noqa: N802
    """functions.py:89-97."""
    return grey_equalize(imgL), grey_equalize(imgR)


# ---------------------------------------------------------------------------
# functions.py:104-128
# ---------------------------------------------------------------------------
def _pair(grayL, grayR):
    L = _u8(grayL, "grayL", 2)
    R = _u8(grayR, "grayR", 2)
    if L.shape != R.shape:
        raise ValueError(f"left {L.shape} and right {R.shape} images differ in size")
    return L, R


def sgbm_compute(grayL, grayR, params=None):
    """stereoProcessor.compute(grayL, grayR): (H, W) int16 disparity x16."""
    L, R = _pair(grayL, grayR)
    H, W = L.shape
    prm = params or _processor_params()
    out = np.empty((H, W), np.int16)
    _abi.call("sv_sgbm_compute", _abi.ptr(L), _abi.ptr(R), H, W, ctypes.byref(prm), _abi.ptr(out))
    return out


def filterSpeckles(img, newVal, maxSpeckleSize, maxDiff, buf=None):  # noqa: N802
    """cv2.filterSpeckles on an int16 image, in place; returns (img, buf) like cv2."""
    if not isinstance(img, np.ndarray) or img.dtype != np.int16 or img.ndim != 2:
        raise TypeError("filterSpeckles expects a 2-D int16 numpy array")
    work = img if img.flags.c_contiguous else np.ascontiguousarray(img)
    _abi.call("sv_filter_speckles", _abi.ptr(work), work.shape[0], work.shape[1], int(newVal), int(maxSpeckleSize),
              int(maxDiff))
    if work is not img:
        img[...] = work
    return img, buf


def stereo_disparity(grayL, grayR, max_disparity=128, crop_disparity=False, params=None, with_raw=False):
    """Array form of functions.disparity; with_raw also returns the int16 SGBM
    result before and after filterSpeckles."""
    L, R = _pair(grayL, grayR)
    H, W = L.shape
    prm = params or _processor_params()
    rows, cols = (min(390, H), max(W - 135, 0)) if crop_disparity else (H, W)
    out = np.empty((rows, cols), np.uint8)
    raw = np.empty((H, W), np.int16) if with_raw else None
    filt = np.empty((H, W), np.int16) if with_raw else None
    _abi.call("sv_disparity", _abi.ptr(L), _abi.ptr(R), H, W, ctypes.byref(prm), int(max_disparity),
              int(bool(crop_disparity)), _abi.ptr(out), _abi.ptr(raw), _abi.ptr(filt))
    return (out, raw, filt) if with_raw else out


def disparity(grayL, grayR, max_disparity, crop_disparity):
    """functions.py:104-128 on the GPU."""
    return stereo_disparity(grayL, grayR, max_disparity, crop_disparity)
