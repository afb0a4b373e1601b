"""The reference's per-frame loop over a sequence of device batches, software-pipelined (sv_loop_*).

loop.py:59-78 calls performStereoVision (stereovision.py:26-247) once per frame. On the device the frames come
in batches and every batch runs the non-cv2 stages of that function:

    input -> pre-pass (fillDisparity / fillAltDisparity, carmask)      stereovision.py:53-76
          -> maskpoints (masked step-2 projection)                      stereovision.py:74-85
          -> RANSAC(maskpoints, 600), frame g seeded with seed_base + g stereovision.py:94
             (two stages: the draw replay, the evaluation)
          -> the pipeline with each frame's own plane                   stereovision.py:97-113
          -> road raster + non-zero walk (+ imageRoadMap)               stereovision.py:131-156

FrameLoop keeps `slots` batches in flight, one HIP stream each; a stage of batch k waits for the same stage of
batch k - 1 (a device event), and the RANSAC evaluation of batch k for batch k - 1's road pass, so with two slots
batch k + 1's draw — one wave's dependent chain per frame, the HBM nearly idle — runs beside batch k's HBM-bound
pipeline and road pass, and batch k + 1's evaluation (a CU's LDS per frame) beside batch k + 2's pre-pass. The previous cleaned frame of
fillDisparity is carried from batch to batch on the device: a sequence of batches gives exactly the results of
one long batch (tests/test_gpu_loop.py checks every frame against tests/golden/plane_digests.npz).

    loop = FrameLoop(4096, carmask=mask)
    for i in range(n):
        seq = loop.submit(i * 4096)          # synthetic frames of global ids i*4096.. (source="synth")
        ...                                  # the host returns while the GPU works on the batches in flight
    loop.wait(seq)
    b, first = loop.batch(seq)               # a Batch: read_points / read_road / read_ransac / digest ...
"""
import ctypes
import weakref

import numpy as np

from . import _abi
from .batch import CAMERA, Batch

STAGES = ("input", "prepass", "maskpoints", "draw", "eval", "pipeline", "road")
_SOURCES = {"caller": 0, "synth": 1}
_PREPASS = {"none": 0, "previous": 1, "mean": 2}
_ROAD = {"none": 0, "walk": 1, "map": 2}


class FrameLoop:
    def __init__(self, frames, H=544, W=1024, step=1, slots=2, source="synth", prepass="previous", trials=600,
                 k=600, seed_base=0, point_thr=0.05, hist_thr=10, road="walk", carmask=None, camera=None,
                 device=0):
        self.frames, self.H, self.W, self.step, self.slots, self.device = frames, H, W, step, slots, device
        prm = _abi.LoopParams(frames=frames, H=H, W=W, step=step, slots=slots, source=_SOURCES[source],
                              prepass=_PREPASS[prepass], trials=trials, k=k, seed_base=seed_base,
                              point_thr=float(point_thr), hist_thr=int(hist_thr), road=_ROAD[road])
        m = None
        if carmask is not None:
            m = np.ascontiguousarray(carmask, np.uint8)
            if m.shape != (H, W):
                raise ValueError(f"carmask shape {m.shape} != {(H, W)}")
        h = ctypes.c_void_p()
        _abi.call("sv_loop_create", device, ctypes.byref(prm), ctypes.byref(camera or CAMERA), _abi.ptr(m),
                  ctypes.byref(h))
        self._h = h
        self._views = weakref.WeakSet()   # the Batch views handed out: invalidated by close()

    def _view(self, handle):
        v = Batch._view(handle, self.frames, self.H, self.W, self.step, self.device)
        self._views.add(v)
        return v

    def acquire(self):
        """The Batch the next submit() runs (source="caller": fill it first, e.g. upload() or sgbm(); the slot keeps
        the frames written into it — the pre-pass writes the cleaned frames elsewhere — so a slot submitted again
        without refilling processes the same raw frames)."""
        out = ctypes.c_void_p()
        _abi.call("sv_loop_acquire", self._h, ctypes.byref(out))
        return self._view(out.value)

    def submit(self, first_frame_id):
        """Enqueue the next batch (global frame ids first_frame_id..) through every stage; its sequence number."""
        seq = ctypes.c_int64(0)
        _abi.call("sv_loop_submit", self._h, int(first_frame_id), ctypes.byref(seq))
        return seq.value

    def wait(self, seq):
        _abi.call("sv_loop_wait", self._h, int(seq))

    def batch(self, seq):
        """(Batch, first global frame id) holding batch seq's results (until seq + slots is acquired/submitted)."""
        out = ctypes.c_void_p()
        first = ctypes.c_int64(0)
        _abi.call("sv_loop_batch", self._h, int(seq), ctypes.byref(out), ctypes.byref(first))
        return self._view(out.value), first.value

    def timeline(self, seq):
        """{stage: (start_ms, end_ms)} of batch seq, ms since the loop's first submit (device events)."""
        out = np.zeros(2 * len(STAGES), np.float64)
        _abi.call("sv_loop_timeline", self._h, int(seq), _abi.ptr(out))
        return {name: (float(out[2 * i]), float(out[2 * i + 1])) for i, name in enumerate(STAGES)}

    def close(self):
        if self._h:
            # a view the caller kept must not reach the destroyed slots: its handle becomes NULL, so a later call
            # on it raises SvxError ("null batch") instead of touching freed memory
            for v in list(getattr(self, "_views", ())):
                v._h = None
            _abi.call("sv_loop_destroy", self._h)
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
