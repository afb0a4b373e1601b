"""Batched, device-resident API.

Frames live in HBM for their whole life: generated on the device by the
counter-based synthetic generator (or uploaded once), projected by K1 into
dense fp32 X/Y/Z planes, or run through the plane/hue/compaction pipeline.
Only the small per-frame results are copied back, on request.
"""
import ctypes

import numpy as np

from . import _abi
from .dropin import DEFAULT_CAMERA

CAMERA = _abi.Camera(*DEFAULT_CAMERA)


def synthetic_plane(f=DEFAULT_CAMERA[0], B=DEFAULT_CAMERA[1], ch=DEFAULT_CAMERA[3], horizon=200):
    """SURVEY §8d plane matching the synthetic road (a*X + b*Y + c*Z = 1)."""
    k = 0.6
    return (0.0, k / B, -k * (horizon - ch) / (f * B))


_WHICH = {"project": 0, "pipeline": 1, "sgbm": 2}


class Batch:
    """`frames` x H x W disparity (+BGR) frames resident on one GPU."""

    def __init__(self, frames, H=544, W=1024, step=1, with_bgr=True, with_points=False, device=0):
        h = ctypes.c_void_p()
        _abi.call("sv_batch_create", device, frames, H, W, step, int(with_bgr), int(with_points),
                  ctypes.byref(h))
        self._h = h
        self._owned = True
        self._init_info(frames, H, W, step, device)

    def _init_info(self, frames, H, W, step, device):
        self.frames, self.H, self.W, self.step, self.device = frames, H, W, step, device
        info = np.zeros(8, np.int64)
        _abi.call("sv_batch_info", self._h, _abi.ptr(info))
        self.Hg, self.Wg, self.pitch, self.Ng = (int(v) for v in info[:4])

    @classmethod
    def _view(cls, handle, frames, H, W, step, device):
        """A Batch over a handle some other object owns (a FrameLoop slot): never destroyed by this object."""
        b = cls.__new__(cls)
        b._h = ctypes.c_void_p(handle)
        b._owned = False
        b._init_info(frames, H, W, step, device)
        return b

    # -- lifetime ---------------------------------------------------------------
    def close(self):
        if self._h and self._owned:
            _abi.call("sv_batch_destroy", self._h)
        self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    # -- inputs -------------------------------------------------------------------
    def synth(self, first_frame_id=0):
        _abi.call("sv_batch_synth", self._h, int(first_frame_id))

    def upload(self, frame, disp, bgr=None):
        disp = np.ascontiguousarray(disp, np.uint8)
        if disp.shape != (self.H, self.W):
            raise ValueError(f"disp shape {disp.shape} != {(self.H, self.W)}")
        if bgr is not None:
            bgr = np.ascontiguousarray(bgr, np.uint8)
            if bgr.shape != (self.H, self.W, 3):
                raise ValueError(f"bgr shape {bgr.shape} != {(self.H, self.W, 3)}")
        _abi.call("sv_batch_upload", self._h, frame, _abi.ptr(disp), _abi.ptr(bgr))

    def tune(self, qpl=1, nontemporal=1):
        """K1 launch shape: quads per lane (1, 2, 4) and non-temporal stores."""
        _abi.call("sv_batch_tune", self._h, int(qpl), int(nontemporal))

    PIPE_MODES = {"auto": 0, "tiled": 1, "resident": 2, "resident_nopf": 3, "resident_pf2": 4}

    def pipeline_mode(self, mode="auto"):
        """Pipeline kernel family: "auto", "tiled" (tiles across workgroups) or
        "resident" (one workgroup per frame). Results are identical."""
        _abi.call("sv_batch_pipeline_mode", self._h, self.PIPE_MODES[mode])

    PREPASS = {"none": 0, "previous": 1, "mean": 2}

    def set_mask(self, mask):
        """Grey carmask (H x W uint8) for the pre-pass's masked disparity; None clears it."""
        m = None if mask is None else np.ascontiguousarray(mask, np.uint8)
        if m is not None and m.shape != (self.H, self.W):
            raise ValueError(f"mask shape {m.shape} != {(self.H, self.W)}")
        _abi.call("sv_batch_set_mask", self._h, _abi.ptr(m))

    def prepass(self, option="previous", prev0=None, sync=True):
        """stereovision.py:53-76 over the batch's frames in order (see sv_batch_prepass)."""
        p0 = None if prev0 is None else np.ascontiguousarray(prev0, np.uint8)
        _abi.call("sv_batch_prepass", self._h, self.PREPASS[option], _abi.ptr(p0), int(sync))

    def read_disp(self, frame, masked=False):
        d = np.empty((self.H, self.W), np.uint8)
        m = np.empty((self.H, self.W), np.uint8) if masked else None
        _abi.call("sv_batch_read_disp", self._h, frame, _abi.ptr(d), _abi.ptr(m))
        return (d, m) if masked else d

    # -- compute -------------------------------------------------------------------
    def project(self, camera=None, sync=True):
        cam = camera or CAMERA
        _abi.call("sv_batch_project", self._h, ctypes.byref(cam), int(sync))

    def pipeline(self, plane=None, point_thr=0.05, hist_thr=10, camera=None, chunk=0, sync=True):
        cam = camera or CAMERA
        pl = _abi.Plane(*(plane if plane is not None else synthetic_plane()))
        _abi.call("sv_batch_pipeline", self._h, ctypes.byref(cam), ctypes.byref(pl), float(point_thr),
                  int(hist_thr), int(chunk), int(sync))

    def pipeline_planes(self, point_thr=0.05, hist_thr=10, camera=None, chunk=0, sync=True):
        """The pipeline with each frame's own RANSAC plane (after ransac()); no plane -> no points."""
        cam = camera or CAMERA
        _abi.call("sv_batch_pipeline_planes", self._h, ctypes.byref(cam), float(point_thr), int(hist_thr),
                  int(chunk), int(sync))

    def pipeline_dev(self, dplane, point_thr=0.05, hist_thr=10, camera=None, chunk=0, sync=True):
        """The pipeline with the plane in device memory (a device pointer to a, b, c
        on this batch's device, e.g. RcclComm.broadcast_plane_dev's): no host copy."""
        cam = camera or CAMERA
        _abi.call("sv_batch_pipeline_dev", self._h, ctypes.byref(cam), ctypes.c_void_p(dplane), float(point_thr),
                  int(hist_thr), int(chunk), int(sync))

    def read_frame_plane(self, frame):
        """(a, b, c, |abc|) of the frame's plane as the kernels use it; |abc| = -1 without a plane."""
        out = np.empty(4, np.float64)
        _abi.call("sv_batch_read_frame_plane", self._h, frame, _abi.ptr(out))
        return out

    def sync(self):
        _abi.call("sv_batch_sync", self._h)

    # -- disparity stage (functions.py:104-128) ------------------------------------
    def pair_shape(self, H, W):
        """The stereo pairs' shape: the batch's own (default), or an H x W pair
        whose crop_disparity=True output [0:390, 135:W] is the batch
        (functions.py:122-124)."""
        _abi.call("sv_batch_pair_shape", self._h, int(H), int(W))
        self._pair = (int(H), int(W))

    def upload_bgr_pair(self, frame, left, right):
        """One host BGR stereo pair (the pair shape x 3), for preprocess()."""
        shape = getattr(self, "_pair", (self.H, self.W)) + (3,)
        L = np.ascontiguousarray(left, np.uint8)
        R = np.ascontiguousarray(right, np.uint8)
        if L.shape != shape or R.shape != shape:
            raise ValueError(f"BGR pair must be {shape}")
        _abi.call("sv_batch_upload_bgr_pair", self._h, frame, _abi.ptr(L), _abi.ptr(R))

    def synth_bgr_pair(self, first_frame_id=0):
        """Synthetic BGR stereo pairs for global frame ids first.. (device)."""
        _abi.call("sv_batch_synth_bgr_pair", self._h, int(first_frame_id))

    def preprocess(self, gamma=1.4, sync=True):
        """stereovision.py:44-46 on the BGR pairs: preProcessImages (gamma,
        applied as the pairs are read: the stored pairs stay raw, so every call
        corrects them once, as cv2.LUT returns new images), greyscale (-> the
        SGBM pairs) and the corrected left image's colours into the batch
        (with_bgr)."""
        from .disparity import gamma_table
        lut = np.ascontiguousarray(gamma_table(gamma), np.uint8)
        _abi.call("sv_batch_preprocess", self._h, _abi.ptr(lut), int(bool(sync)))

    def synth_pair(self, first_frame_id=0):
        """Synthetic rectified grey pairs for global frame ids first.. (device)."""
        _abi.call("sv_batch_synth_pair", self._h, int(first_frame_id))

    def upload_pair(self, frame, left, right):
        L = np.ascontiguousarray(left, np.uint8)
        R = np.ascontiguousarray(right, np.uint8)
        shape = getattr(self, "_pair", (self.H, self.W))
        if L.shape != shape or R.shape != shape:
            raise ValueError(f"pair must be {shape[0]}x{shape[1]}")
        _abi.call("sv_batch_upload_pair", self._h, frame, _abi.ptr(L), _abi.ptr(R))

    def sgbm(self, max_disparity=128, chunk=0, **params):
        """functions.disparity of every pair -> the batch's disparity (cropped
        when pair_shape() set the uncropped pair shape)."""
        from .disparity import sgbm_params
        prm = sgbm_params(**params)
        _abi.call("sv_batch_sgbm", self._h, ctypes.byref(prm), int(max_disparity), int(chunk))

    def last_ms(self, which="project"):
        ms = ctypes.c_float(0)
        _abi.call("sv_batch_last_ms", self._h, _WHICH[which], ctypes.byref(ms))
        return float(ms.value)

    def timing(self, which="project"):
        """(total_ms, launches) of the per-launch event timings since reset_timing()."""
        tot = ctypes.c_double(0)
        cnt = ctypes.c_int64(0)
        _abi.call("sv_batch_timing", self._h, _WHICH[which], ctypes.byref(tot), ctypes.byref(cnt))
        return float(tot.value), int(cnt.value)

    def placement(self, which="project"):
        """The first large call's placement probe: {"tried_ms": [...], "kept": index or None} (which = "project"
        for K1's planes, "pipeline" for the resident pipeline's output planes, "sgbm" for the SGBM cost volumes;
        sv_batch_placement)."""
        ms = (ctypes.c_float * 8)()
        n, kept = ctypes.c_int(0), ctypes.c_int(-1)
        _abi.call("sv_batch_placement", self._h, {"project": 0, "pipeline": 1, "sgbm": 2}[which], ms, 8,
                  ctypes.byref(n), ctypes.byref(kept))
        return {"tried_ms": [round(float(ms[i]), 4) for i in range(n.value)],
                "kept": kept.value if kept.value >= 0 else None}

    def kernel_name(self, which="project"):
        """The kernel instance the last project / pipeline call launched, as rocprofv3 names it
        (sv_batch_kernel_name): a PMC profile under that name measured the kernel this batch timed."""
        buf = ctypes.create_string_buffer(256)
        _abi.call("sv_batch_kernel_name", self._h, _WHICH[which], buf, 256)
        return buf.value.decode()

    def reset_timing(self):
        _abi.call("sv_batch_timing_reset", self._h)

    def road_raster(self, sync=True):
        """generatePointsAsImage of every frame's pipeline points (device)."""
        _abi.call("sv_batch_road_raster", self._h, int(sync))

    def nonzero(self, sync=True):
        """Raster-order non-zero walk of every road image (device)."""
        _abi.call("sv_batch_nonzero", self._h, int(sync))

    def road_map(self, enable=True):
        """Also write stereovision.py:131-133's imageRoadMap (the frame's BGR with [0, 255, 0] at its
        planePoints) in every later road_raster() pass."""
        _abi.call("sv_batch_road_map", self._h, int(bool(enable)))

    def road_bits(self, enable=True):
        """Later resident pipeline calls (1024-wide frames, step 1) also write the bitmap of their points' pixels,
        and road_raster() builds its outputs from it instead of re-reading the points (sv_batch_road_bits)."""
        _abi.call("sv_batch_road_bits", self._h, int(bool(enable)))

    def read_road_map(self, frame):
        out = np.empty((self.H, self.W, 3), np.uint8)
        _abi.call("sv_batch_read_road_map", self._h, frame, _abi.ptr(out))
        return out

    def read_road(self, frame, walk=False):
        img = np.empty((self.H, self.W), np.uint8)
        if not walk:
            _abi.call("sv_batch_read_road", self._h, frame, _abi.ptr(img), None, 0, None)
            return img
        n = ctypes.c_int64(0)
        pts = np.empty((self.Ng, 2), np.int32)
        _abi.call("sv_batch_read_road", self._h, frame, _abi.ptr(img), _abi.ptr(pts), self.Ng, ctypes.byref(n))
        return img, pts[: n.value]

    def ransac(self, seed_base, trials, k=600, first_frame=0, camera=None, sync=True):
        """RANSAC(maskpoints, trials) of every frame on the device (stereovision.py:84-94), frame F
        drawing what CPython draws after random.seed(seed_base + first_frame + F)."""
        cam = camera or CAMERA
        _abi.call("sv_batch_ransac", self._h, ctypes.byref(cam), int(seed_base), int(first_frame), int(trials),
                  int(k), int(sync))

    def read_ransac(self, frame):
        """dict(abc (3,) float64, err, trial (-1: none ran), flags) of one frame."""
        abc = np.empty(3, np.float64)
        err = ctypes.c_double(0)
        trial = ctypes.c_int32(0)
        flags = ctypes.c_uint32(0)
        _abi.call("sv_batch_read_ransac", self._h, frame, _abi.ptr(abc), ctypes.byref(err), ctypes.byref(trial),
                  ctypes.byref(flags))
        return dict(abc=abc, err=float(err.value), trial=int(trial.value), flags=int(flags.value))

    def ransac_trace(self, trials):
        """Record the first `trials` trials' drawn indices per frame in later ransac() calls."""
        _abi.call("sv_batch_ransac_trace", self._h, int(trials))

    def read_ransac_trace(self, frame):
        """(trials, k + 3) int32: each traced trial's sample indices, then P1..P3
        (trials and k of the last ransac() call, as the library recorded them)."""
        t, k = ctypes.c_int(0), ctypes.c_int(0)
        _abi.call("sv_batch_read_ransac_trace", self._h, frame, None, 0, ctypes.byref(t), ctypes.byref(k))
        out = np.empty((t.value, k.value + 3), np.int32)
        _abi.call("sv_batch_read_ransac_trace", self._h, frame, _abi.ptr(out), out.size, None, None)
        return out

    def read_maskpoints(self, frame):
        """The frame's maskpoints (n x 3 float64, raster order) as the batched RANSAC saw them."""
        cap = (self.H // 2) * (self.W // 2)
        xyz = np.empty((max(cap, 1), 3), np.float64)
        n = ctypes.c_int64(0)
        _abi.call("sv_batch_read_maskpoints", self._h, frame, _abi.ptr(xyz), cap, ctypes.byref(n))
        return xyz[: n.value]

    DIGEST_FIELDS = ("n_valid", "n_kept", "n_kept2", "disp_hash", "hist_hash", "pts_hash", "bad")

    def digest(self, which="pipeline", camera=None):
        """Per-frame verification digests of the current outputs (which = "dense" for K1's
        planes, "pipeline" for the pipeline's points): a (frames, 8) uint64 array with the
        columns of DIGEST_FIELDS (see sv_batch_digest); computed on the device."""
        cam = camera or CAMERA
        out = np.empty((self.frames, 8), np.uint64)
        _abi.call("sv_batch_digest", self._h, ctypes.byref(cam), 0 if which == "dense" else 1, _abi.ptr(out))
        return out

    # -- outputs -------------------------------------------------------------------
    def read_dense(self, frame):
        shape = (self.Hg, self.pitch)
        X, Y, Z = (np.empty(shape, np.float32) for _ in range(3))
        _abi.call("sv_batch_read_dense", self._h, frame, _abi.ptr(X), _abi.ptr(Y), _abi.ptr(Z))
        return X, Y, Z

    def read_counts(self):
        c = np.empty((self.frames, 3), np.int64)
        _abi.call("sv_batch_read_counts", self._h, _abi.ptr(c))
        return c

    def read_hist(self, frame):
        h = np.empty(1024, np.uint32)
        _abi.call("sv_batch_read_hist", self._h, frame, _abi.ptr(h))
        return h

    def read_points(self, frame):
        n = ctypes.c_int64(0)
        cap = self.Ng
        xyz = np.empty((cap, 3), np.float32)
        pts = np.empty((cap, 2), np.int32)
        _abi.call("sv_batch_read_points", self._h, frame, _abi.ptr(xyz), _abi.ptr(pts), cap, ctypes.byref(n))
        k = n.value
        return xyz[:k], pts[:k]


def pipeline_frame(disp, bgr, step=2, plane=None, point_thr=0.05, hist_thr=10, camera=None):
    """Fused chain for one host frame (sv_pipeline_frame). Returns dict like the oracle."""
    disp = np.ascontiguousarray(disp, np.uint8)
    bgr = np.ascontiguousarray(bgr, np.uint8)
    H, W = disp.shape
    hg = (H - 1 + step - 1) // step
    wg = (W - 1 + step - 1) // step
    cap = max(hg * wg, 1)
    counts = np.zeros(3, np.int64)
    hist = np.zeros(1024, np.uint32)
    xyz = np.empty((cap, 3), np.float32)
    pts = np.empty((cap, 2), np.int32)
    cam = camera or CAMERA
    pl = _abi.Plane(*(plane if plane is not None else synthetic_plane()))
    _abi.call("sv_pipeline_frame", _abi.ptr(disp), _abi.ptr(bgr), H, W, step, ctypes.byref(cam),
              ctypes.byref(pl), float(point_thr), int(hist_thr), _abi.ptr(counts), _abi.ptr(hist),
              _abi.ptr(xyz), _abi.ptr(pts), cap)
    n2 = int(counts[2])
    return dict(counts=tuple(int(v) for v in counts), hist=hist, xyz2=xyz[:n2], pts=pts[:n2])


def hue_lut(device=0, variant=0):
    """The device's hue bin of every colour R << 16 | G << 8 | B: variant 0 the exact function, 1 the resident
    pipeline's fp32 path (sv_hue_lut_variant)."""
    lut = np.empty(1 << 24, np.int16)
    _abi.call("sv_hue_lut_variant", device, int(variant), _abi.ptr(lut))
    return lut


def delta_tables(H=544, W=1024, camera=None, device=0):
    dx = np.empty((256, W), np.int8)
    dy = np.empty((256, H), np.int8)
    cam = camera or CAMERA
    _abi.call("sv_delta_tables", device, H, W, ctypes.byref(cam), _abi.ptr(dx), _abi.ptr(dy))
    return dx, dy


def synth_frame(frame_id, H=544, W=1024, device=0):
    disp = np.empty((H, W), np.uint8)
    bgr = np.empty((H, W, 3), np.uint8)
    _abi.call("sv_synth_frame", device, int(frame_id), H, W, _abi.ptr(disp), _abi.ptr(bgr))
    return disp, bgr
