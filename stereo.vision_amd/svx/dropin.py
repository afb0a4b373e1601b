"""Drop-in replacements for the reference's hot-path functions.

The reference (thien/stereo.vision) has no plugin/FFI API: stereovision.py
does ``import functions as f`` (stereovision.py:3) and resolves
``f.projectDisparityTo3d`` etc. at call time (stereovision.py:84-111). The
boundary is therefore the attributes of the ``functions`` module:

    import functions, svx.dropin
    svx.dropin.install(functions)      # loop.py / single_frame.py then run unchanged

Signatures, argument meaning, return conventions and error behaviour follow the
reference:

* ``projectDisparityTo3d(disparity, max_disparity, rgb=[])`` (functions.py:178-198):
  ``max_disparity`` is accepted and ignored (as in the reference); ``rgb`` is
  used iff ``len(rgb) > 0``. Returns a Sequence (``random.sample`` in RANSAC
  needs one, functions.py:252,286; svx/points.py: rows made when first read, a
  plain list after a mutation) of rows supporting ``row[0..5]``
  and ``row[:3]``; XYZ are ``np.float64`` bit-identical to the reference and
  R,G,B are numpy scalars (np.float64), which keeps ``BGRtoHSVHue`` keys
  identical (Python ints would not: SURVEY §0 trap 3).
* ``project3DPointsTo2DImagePoints(points)`` (functions.py:201-209): returns
  an (N, 2) float64 array that ``np.array(.., np.int32).reshape((-1,1,2))``
  (stereovision.py:112-113) accepts, (0, 2) for no points.
* ``generatePointsAsImage(points)`` (functions.py:339-344): grey road image;
  ``nonzero_points(img)`` gives sanitiseRoadImage's final pixel walk.
* ``RANSAC(points, trials)`` (functions.py:278-298): see svx/ransac.py — same
  draws from the global ``random`` stream, trials on the GPU, same plane bits.
* ``calculatePointErrors``, ``computePlanarThreshold``,
  ``calculateColourHistogram``, ``filterPointsByHistogram`` (functions.py:
  212-230, :300-323): see svx/stages.py — one device call each, same return
  types, dict order and errors as the reference.
* disparity stage (functions.py:61-128): ``gammaChange``, ``preProcessImages``,
  ``greyscale`` and ``disparity`` (StereoSGBM + filterSpeckles + scaling) —
  see svx/disparity.py.
* disparity pre-pass (functions.py:141-172): ``fillDisparity`` (new array, or
  the input itself when there is no previous frame), ``fillAltDisparity`` (in
  place, returns its argument), ``maskDisparity`` (new array; the mask is the
  installed module's ``carmask``, functions.py:35) and ``capDisparity`` (returns
  its argument: the reference discards the masked result, functions.py:164-167).

Failures raise ``RuntimeError`` (``SvxError``), which the reference's own
``try/except`` at stereovision.py:92-126 handles like any reference error.
"""
import ctypes

import numpy as np

from . import _abi

# functions.py:15,19,21,22
DEFAULT_CAMERA = (399.9745178222656, 0.2090607502, 474.5, 262.0)
REFERENCE_STEP = 2   # functions.py:185-186 hard-codes the grid step

_module = None       # the installed `functions` module (its constants are read per call)


def _camera():
    if _module is not None:
        m = _module
        return _abi.Camera(m.camera_focal_length_px, m.stereo_camera_baseline_m,
                           m.image_centre_w, m.image_centre_h)
    return _abi.Camera(*DEFAULT_CAMERA)


def _as_u8(a, ndim, what):
    arr = np.asarray(a)
    if arr.dtype != np.uint8:
        raise TypeError(f"{what} must be uint8 (as functions.disparity / cv2.imread produce), got {arr.dtype}")
    if arr.ndim != ndim:
        raise ValueError(f"{what} must have {ndim} dimensions, got shape {arr.shape}")
    if arr.strides[-1] != arr.itemsize or (ndim == 3 and arr.strides[1] != 3):
        arr = np.ascontiguousarray(arr)
    return arr


def project_frame(disparity, rgb=None, step=REFERENCE_STEP, camera=None):
    """Array form: (xyz (N,3) float64, rgb (N,3) uint8 or None) in reference order."""
    disp = _as_u8(disparity, 2, "disparity")
    h, w = disp.shape
    bgr = None
    if rgb is not None and len(rgb) > 0:
        bgr = _as_u8(rgb, 3, "rgb")
        if bgr.shape[0] < h or bgr.shape[1] < w or bgr.shape[2] < 3:
            raise IndexError(f"rgb shape {bgr.shape} smaller than disparity {disp.shape}")
        if bgr.shape[2] != 3:
            bgr = np.ascontiguousarray(bgr[:, :, :3])
    hg = (h - 1 + step - 1) // step if h > 1 else 0
    wg = (w - 1 + step - 1) // step if w > 1 else 0
    cap = max(hg * wg, 1)
    xyz = np.empty((cap, 3), np.float64)
    out_rgb = np.empty((cap, 3), np.uint8) if bgr is not None else None
    n = ctypes.c_int64(0)
    cam = camera if camera is not None else _camera()
    _abi.call("sv_project_frame", _abi.ptr(disp), h, w, disp.strides[0],
              _abi.ptr(bgr), bgr.strides[0] if bgr is not None else 0, step, ctypes.byref(cam),
              _abi.ptr(xyz), _abi.ptr(out_rgb), cap, ctypes.byref(n))
    k = n.value
    return xyz[:k], (out_rgb[:k] if out_rgb is not None else None)


from .points import PointList, as_points_array, gather_columns  # noqa: E402,F401  (re-exported)


def project_rows(disparity, rgb=None, step=REFERENCE_STEP, camera=None):
    """(N, 6) float64 rows X, Y, Z, R, G, B — or (N, 3) without colours — in reference order, laid out on the
    device and copied straight into pooled page-locked memory (sv_project_rows, one DMA, no host assembly)."""
    disp = _as_u8(disparity, 2, "disparity")
    h, w = disp.shape
    bgr = None
    if rgb is not None and len(rgb) > 0:
        bgr = _as_u8(rgb, 3, "rgb")
        if bgr.shape[0] < h or bgr.shape[1] < w or bgr.shape[2] < 3:
            raise IndexError(f"rgb shape {bgr.shape} smaller than disparity {disp.shape}")
        if bgr.shape[2] != 3:
            bgr = np.ascontiguousarray(bgr[:, :, :3])
    cols = 6 if bgr is not None else 3
    hg = (h - 1 + step - 1) // step if h > 1 else 0
    wg = (w - 1 + step - 1) // step if w > 1 else 0
    cap = max(hg * wg, 1)
    cam = camera if camera is not None else _camera()
    n = ctypes.c_int64(0)
    if hg * wg == 0:
        rows = np.empty((cap, cols), np.float64)
    else:
        rows = _abi.pinned_empty((cap, cols), np.float64)
    _abi.call("sv_project_rows", _abi.ptr(disp), h, w, disp.strides[0], _abi.ptr(bgr),
              bgr.strides[0] if bgr is not None else 0, step, ctypes.byref(cam), _abi.ptr(rows), cols, cap,
              ctypes.byref(n))
    return rows[: n.value]


def projectDisparityTo3d(disparity, max_disparity, rgb=[]):  # noqa: N802,B006 (reference signature)
    """functions.py:178-198 on the GPU. Returns a Sequence of rows (see module doc)."""
    return PointList(project_rows(disparity, rgb))


def project3DPointsTo2DImagePoints(points):  # noqa: N802
    """functions.py:201-209 on the GPU: (N,2) float64 [x, y]."""
    n = len(points)
    if n == 0:
        return np.zeros((0, 2), np.float64)
    arr = gather_columns(points, 0, 3, pinned=True)   # X, Y, Z only (a selection: one C pass, svx/points.py)
    if arr.ndim != 2 or arr.shape[1] < 3:
        raise ValueError(f"points must be rows of at least [X, Y, Z], got shape {arr.shape}")
    out = _abi.pinned_empty((n, 2), np.float64)   # page-locked: the device-to-host copy is a direct DMA
    cam = _camera()
    _abi.call("sv_backproject", _abi.ptr(arr), n, arr.shape[1], ctypes.byref(cam), _abi.ptr(out))
    return out


# ---------------------------------------------------------------------------
# disparity pre-pass (functions.py:141-172)
# ---------------------------------------------------------------------------
def fill_previous(disparity, previous):
    """Array form of fillDisparity: d > 2 ? d : min(255, d + prev)."""
    disp = _as_u8(disparity, 2, "disparity")
    prev = _as_u8(previous, 2, "previousDisparity")
    if prev.shape != disp.shape:
        raise ValueError(f"previousDisparity shape {prev.shape} != disparity shape {disp.shape}")
    out = np.empty_like(disp)
    _abi.call("sv_fill_previous", _abi.ptr(disp), _abi.ptr(prev), disp.shape[0], disp.shape[1], _abi.ptr(out))
    return out


def fillDisparity(disparity, previousDisparity):  # noqa: N802
    """functions.py:141-148 on the GPU."""
    if previousDisparity is None:
        return disparity
    return fill_previous(disparity, previousDisparity)


def fillAltDisparity(disparity):  # noqa: N802
    """functions.py:150-162 on the GPU: in place (like the reference), returns its argument."""
    if not isinstance(disparity, np.ndarray) or disparity.dtype != np.uint8 or disparity.ndim != 2:
        raise TypeError("fillAltDisparity expects a 2-D uint8 numpy array")
    work = np.ascontiguousarray(disparity).copy() if not disparity.flags.c_contiguous else disparity
    _abi.call("sv_fill_mean", _abi.ptr(work), work.shape[0], work.shape[1])
    if work is not disparity:
        disparity[...] = work
    return disparity


def mask_disparity(disparity, mask):
    """Array form of maskDisparity with an explicit grey mask: mask != 0 ? d : 0."""
    disp = _as_u8(disparity, 2, "disparity")
    m = _as_u8(mask, 2, "mask")
    if m.shape != disp.shape:
        raise ValueError(f"mask shape {m.shape} != disparity shape {disp.shape}")
    out = np.empty_like(disp)
    _abi.call("sv_mask_disparity", _abi.ptr(disp), _abi.ptr(m), disp.shape[0], disp.shape[1], _abi.ptr(out))
    return out


def maskDisparity(disparity):  # noqa: N802
    """functions.py:169-172 on the GPU, with the installed module's carmask."""
    if _module is None or getattr(_module, "carmask", None) is None:
        raise RuntimeError("maskDisparity needs the reference's carmask: install(functions) first "
                           "(or call mask_disparity(disparity, mask))")
    return mask_disparity(disparity, _module.carmask)


def capDisparity(disparity):  # noqa: N802
    """functions.py:164-167: the reference computes a masked copy and discards it,
    returning its argument; so does this (no device work)."""
    return disparity


# ---------------------------------------------------------------------------
# road raster (functions.py:339-344) and the non-zero walk (functions.py:359-365)
# ---------------------------------------------------------------------------
def road_raster(points, shape=(544, 1024)):
    """Array form of generatePointsAsImage: (H, W) uint8, 255 at each [x, y]."""
    p = np.ascontiguousarray(np.asarray(points).reshape(-1, 2), dtype=np.int32)
    H, W = shape
    img = np.empty((H, W), np.uint8)
    try:
        _abi.call("sv_road_raster", _abi.ptr(p), len(p), H, W, _abi.ptr(img))
    except _abi.SvxError as e:
        if "index out of range" in str(e):
            raise IndexError(str(e)) from None
        raise
    return img


def generatePointsAsImage(points):  # noqa: N802
    """functions.py:339-344 on the GPU: the installed module's blackImg shape (the
    reference copies that black image), 544 x 1024 otherwise."""
    black = getattr(_module, "blackImg", None) if _module is not None else None
    shape = black.shape[:2] if black is not None else (544, 1024)
    return road_raster(points, shape)


def nonzero_points(img):
    """The pixel walk that ends sanitiseRoadImage (functions.py:359-365):
    (K, 2) int32 [j, i] of the non-zero pixels in raster order."""
    im = _as_u8(img, 2, "image")
    H, W = im.shape
    out = np.empty((max(H * W, 1), 2), np.int32)
    n = ctypes.c_int64(0)
    _abi.call("sv_nonzero_points", _abi.ptr(im), H, W, _abi.ptr(out), H * W, ctypes.byref(n))
    return out[: n.value]


# snake_case names used by BASELINE.json
project_disparity_to_3d = projectDisparityTo3d
project_3D_points_to_2D = project3DPointsTo2DImagePoints

from .ransac import RANSAC  # noqa: E402  (functions.py:278-298)
from .stages import (calculateColourHistogram, calculatePointErrors, computePlanarThreshold,  # noqa: E402,F401
                     filterPointsByHistogram)
from .disparity import disparity, gammaChange, greyscale, preProcessImages  # noqa: E402,F401 (functions.py:61-128)
from .io import getImagePaths, loadImages  # noqa: E402,F401 (functions.py:41-55, PNG ingest without cv2)

# Functions whose GPU results are pinned against the reference itself (fixtures made by running the reference's
# own code, tests/golden/): installed by default.
PINNED = ("projectDisparityTo3d", "project3DPointsTo2DImagePoints", "fillAltDisparity", "capDisparity",
          "generatePointsAsImage", "RANSAC", "calculatePointErrors", "computePlanarThreshold",
          "calculateColourHistogram", "filterPointsByHistogram", "gammaChange", "preProcessImages")
# Functions that restate OpenCV calls (cv2 is absent here, so nothing pins them to the reference's OpenCV 3.x):
# StereoSGBM + filterSpeckles (functions.py:104-128), cvtColor + equalizeHist (:88-96), cv2.threshold / bitwise /
# add (:140-147), bitwise_and with the carmask (:169-171) and cv2.imread's PNG decode behind getImagePaths /
# loadImages (:41-55; lossless, but OpenCV's channel handling is restated, svx/io.py). Installed only on request
# (install(.., unpinned=True)).
UNPINNED = ("disparity", "greyscale", "fillDisparity", "maskDisparity", "getImagePaths", "loadImages")
PATCHED = PINNED + UNPINNED
ALIASES = {"project_disparity_to_3d": "projectDisparityTo3d",
           "project_3D_points_to_2D": "project3DPointsTo2DImagePoints"}
_saved = {}
_ABSENT = object()


def install(functions_module, unpinned=False):
    """Patch the reference's `functions` module in place (stereovision.py resolves
    f.<name> at call time, so performStereoVision picks the GPU path up).

    By default only the PINNED functions are replaced: the ones whose outputs equal the
    reference's own on its fixtures. unpinned=True also replaces the UNPINNED ones, the
    restatements of OpenCV (SGBM, grey + equalizeHist, fillDisparity, maskDisparity, and
    getImagePaths / loadImages: cv2.imread of the PNG pairs, svx.io) whose equality with the
    reference's cv2 cannot be checked here."""
    global _module
    _abi.lib()  # fail loudly now if libsvx is missing
    _module = functions_module
    names = PINNED + (UNPINNED if unpinned else ()) + tuple(ALIASES)
    for name in names:
        if name not in _saved:
            _saved[name] = getattr(functions_module, name, _ABSENT)
        setattr(functions_module, name, globals()[ALIASES.get(name, name)])
    return functions_module


def uninstall():
    """Restore the attributes install() replaced."""
    global _module
    if _module is not None:
        for name, fn in _saved.items():
            if fn is _ABSENT:
                if hasattr(_module, name):
                    delattr(_module, name)
            else:
                setattr(_module, name, fn)
    _saved.clear()
    _module = None
