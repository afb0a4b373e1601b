"""ctypes binding of libsvx.so (include/svx.h).

The product has exactly one compute path: the hand-written gfx950 kernels in
libsvx.so. If the library is missing or has no device, every call raises —
there is deliberately no CPU fallback.
"""
import ctypes
import os

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "_lib", "libsvx.so")

SV_UNIQUE_ID_BYTES = 128


class SvxError(RuntimeError):
    """A libsvx call failed (message from sv_last_error())."""


class Camera(ctypes.Structure):
    _fields_ = [("f", ctypes.c_double), ("B", ctypes.c_double),
                ("cw", ctypes.c_double), ("ch", ctypes.c_double)]


class Plane(ctypes.Structure):
    _fields_ = [("a", ctypes.c_double), ("b", ctypes.c_double), ("c", ctypes.c_double)]


class LoopParams(ctypes.Structure):
    """sv_loop_params (include/svx.h)."""
    _fields_ = [("frames", ctypes.c_int), ("H", ctypes.c_int), ("W", ctypes.c_int), ("step", ctypes.c_int),
                ("slots", ctypes.c_int), ("source", ctypes.c_int), ("prepass", ctypes.c_int),
                ("trials", ctypes.c_int), ("k", ctypes.c_int), ("seed_base", ctypes.c_uint64),
                ("point_thr", ctypes.c_double), ("hist_thr", ctypes.c_int), ("road", ctypes.c_int)]


P = ctypes.c_void_p
I = ctypes.c_int
I64 = ctypes.c_int64
D = ctypes.c_double
PI64 = ctypes.POINTER(ctypes.c_int64)
PF = ctypes.POINTER(ctypes.c_float)

# name -> argtypes (restype is int unless listed in _RESTYPE)
SIGNATURES = {
    "sv_version": [],
    "sv_last_error": [],
    "sv_device_count": [ctypes.POINTER(I)],
    "sv_init": [I],
    "sv_project_frame": [P, I, I, I64, P, I64, I, ctypes.POINTER(Camera), P, P, I64, PI64],
    "sv_project_rows": [P, I, I, I64, P, I64, I, ctypes.POINTER(Camera), P, I, I64, PI64],
    "sv_host_alloc": [I64, ctypes.POINTER(P)],
    "sv_host_free": [P],
    "sv_backproject": [P, I64, I64, ctypes.POINTER(Camera), P],
    "sv_pipeline_frame": [P, P, I, I, I, ctypes.POINTER(Camera), ctypes.POINTER(Plane), D, I,
                          P, P, P, P, I64],
    "sv_fill_previous": [P, P, I, I, P],
    "sv_fill_mean": [P, I, I],
    "sv_mask_disparity": [P, P, I, I, P],
    "sv_batch_set_mask": [P, P],
    "sv_batch_prepass": [P, I, P, I],
    "sv_batch_read_disp": [P, I, P, P],
    "sv_road_raster": [P, I64, I, I, P],
    "sv_nonzero_points": [P, I, I, P, I64, PI64],
    "sv_batch_road_raster": [P, I],
    "sv_batch_nonzero": [P, I],
    "sv_batch_read_road": [P, I, P, P, I64, PI64],
    "sv_batch_road_map": [P, I],
    "sv_batch_road_bits": [P, I],
    "sv_batch_read_road_map": [P, I, P],
    "sv_point_errors": [P, I64, I64, P, P],
    "sv_hue_histogram": [P, I64, I64, P, P, P],
    "sv_select_less": [P, I64, D, P, PI64],
    "sv_select_bins": [P, I64, P, P, PI64],
    "sv_ransac_draw": [P, P, I64, I64, I, I, P, P, ctypes.POINTER(I)],
    "sv_ransac": [P, P, I64, I64, I, I, P, P, P, P, P, ctypes.POINTER(I)],
    "sv_batch_ransac": [P, ctypes.POINTER(Camera), ctypes.c_uint64, I64, I, I, I],
    "sv_batch_read_ransac": [P, I, P, P, P, P],
    "sv_batch_read_maskpoints": [P, I, P, I64, PI64],
    "sv_batch_ransac_trace": [P, I],
    "sv_batch_read_ransac_trace": [P, I, P, I64, ctypes.POINTER(I), ctypes.POINTER(I)],
    "sv_batch_create": [I, I, I, I, I, I, I, ctypes.POINTER(P)],
    "sv_batch_destroy": [P],
    "sv_batch_info": [P, P],
    "sv_batch_tune": [P, I, I],
    "sv_batch_synth": [P, I64],
    "sv_batch_upload": [P, I, P, P],
    "sv_batch_project": [P, ctypes.POINTER(Camera), I],
    "sv_batch_pipeline": [P, ctypes.POINTER(Camera), ctypes.POINTER(Plane), D, I, I, I],
    "sv_batch_pipeline_mode": [P, I],
    "sv_batch_pipeline_planes": [P, ctypes.POINTER(Camera), D, I, I, I],
    "sv_batch_pipeline_dev": [P, ctypes.POINTER(Camera), P, D, I, I, I],
    "sv_batch_read_frame_plane": [P, I, P],
    "sv_lut_u8": [P, I64, P, P],
    "sv_grey_equalize": [P, I, I, P],
    "sv_sgbm_compute": [P, P, I, I, P, P],
    "sv_filter_speckles": [P, I, I, I, I, I],
    "sv_disparity": [P, P, I, I, P, I, I, P, P, P],
    "sv_batch_pair_shape": [P, I, I],
    "sv_batch_upload_bgr_pair": [P, I, P, P],
    "sv_batch_synth_bgr_pair": [P, I64],
    "sv_batch_preprocess": [P, P, I],
    "sv_batch_synth_pair": [P, I64],
    "sv_batch_upload_pair": [P, I, P, P],
    "sv_batch_sgbm": [P, P, I, I],
    "sv_batch_sync": [P],
    "sv_batch_last_ms": [P, I, PF],
    "sv_batch_timing": [P, I, ctypes.POINTER(D), PI64],
    "sv_batch_timing_reset": [P],
    "sv_batch_placement": [P, I, PF, I, ctypes.POINTER(I), ctypes.POINTER(I)],
    "sv_batch_kernel_name": [P, I, P, I],
    "sv_source_id": [I, P, I],
    "sv_batch_read_dense": [P, I, P, P, P],
    "sv_batch_read_counts": [P, P],
    "sv_batch_read_hist": [P, I, P],
    "sv_batch_read_points": [P, I, P, P, I64, PI64],
    "sv_batch_digest": [P, ctypes.POINTER(Camera), I, P],
    "sv_hue_lut": [I, P],
    "sv_hue_lut_variant": [I, I, P],
    "sv_delta_tables": [I, I, I, ctypes.POINTER(Camera), P, P],
    "sv_synth_frame": [I, I64, I, I, P, P],
    "sv_png_unfilter": [P, I, I, I, P],
    "sv_gather_rgb_u8": [P, I64, I64, P, I64, P],
    "sv_gather_f64": [P, I64, I64, P, I64, I, I, P],
    "sv_loop_create": [I, ctypes.POINTER(LoopParams), ctypes.POINTER(Camera), P, ctypes.POINTER(P)],
    "sv_loop_destroy": [P],
    "sv_loop_acquire": [P, ctypes.POINTER(P)],
    "sv_loop_submit": [P, I64, PI64],
    "sv_loop_wait": [P, I64],
    "sv_loop_batch": [P, I64, ctypes.POINTER(P), PI64],
    "sv_loop_timeline": [P, I64, P],
    "sv_comm_unique_id": [P],
    "sv_comm_init": [I, I, P, I, ctypes.POINTER(P)],
    "sv_comm_destroy": [P],
    "sv_comm_init_all": [I, P, P],
    "sv_comm_group_start": [],
    "sv_comm_group_end": [],
    "sv_comm_broadcast_plane": [P, ctypes.POINTER(Plane), I],
    "sv_comm_broadcast_plane_dev": [P, P, ctypes.POINTER(Plane), I, ctypes.POINTER(P)],
    "sv_multi_pipeline": [I, P, P, ctypes.POINTER(Camera), ctypes.POINTER(Plane), I, D, I, I],
    "sv_comm_allreduce_i64": [P, P, I],
}
_RESTYPE = {"sv_version": ctypes.c_char_p, "sv_last_error": ctypes.c_char_p}

_lib = None


def lib():
    """The loaded libsvx.so (raises ImportError if it was never built)."""
    global _lib
    if _lib is None:
        # SVX_LIB: DIAGNOSTIC A/B only (tools/ab_lib.py times an older build of the
        # library beside this one); symbols that build lacks are left unbound.
        path = os.environ.get("SVX_LIB") or LIB_PATH
        if not os.path.exists(path):
            raise ImportError(f"libsvx.so not found at {path}: build it with "
                              "`python -c 'import __graft_entry__ as g; g.build()'`")
        l = ctypes.CDLL(path)
        for name, args in SIGNATURES.items():
            if path != LIB_PATH and not hasattr(l, name):
                continue
            fn = getattr(l, name)
            fn.argtypes = args
            fn.restype = _RESTYPE.get(name, ctypes.c_int)
        _lib = l
    return _lib


def last_error():
    msg = lib().sv_last_error()
    return msg.decode() if msg else ""


def call(name, *args):
    rc = getattr(lib(), name)(*args)
    if rc != 0:
        raise SvxError(f"{name} failed ({rc}): {last_error()}")
    return rc


def ptr(a):
    """data pointer of a numpy array (or None)."""
    return None if a is None else ctypes.c_void_p(a.ctypes.data)


def device_count():
    n = ctypes.c_int(0)
    rc = lib().sv_device_count(ctypes.byref(n))
    return n.value if rc == 0 else 0


class _PinnedPool:
    """Page-locked host blocks (sv_host_alloc) for drop-in outputs, reused by size class: an array handed out by
    pinned_empty() returns its block here when the array and every view of it are gone, so a frame loop that drops
    each frame's points recycles the same few blocks and every device-to-host copy is a direct DMA."""

    def __init__(self):
        import threading
        self._free = {}
        self._lock = threading.Lock()
        self._closed = False
        self.allocs = 0   # blocks allocated (sv_host_alloc) so far: a steady loop stops adding to it

    def take(self, nbytes):
        size = 1 << max(16, (int(nbytes) - 1).bit_length())   # power-of-two classes from 64 KiB
        with self._lock:
            blocks = self._free.get(size)
            if blocks:
                return blocks.pop(), size
        p = P()
        call("sv_host_alloc", size, ctypes.byref(p))
        self.allocs += 1
        return p.value, size

    def give(self, addr, size):
        if self._closed:
            return
        with self._lock:
            self._free.setdefault(size, []).append(addr)

    def close(self):   # interpreter exit: the HIP runtime may already be gone, so the blocks are left to it
        self._closed = True


_pool = _PinnedPool()


def pinned_empty(shape, dtype):
    """An uninitialised numpy array in pooled page-locked host memory (see _PinnedPool)."""
    import weakref

    import numpy as np
    dt = np.dtype(dtype)
    count = int(np.prod(shape))
    nbytes = max(count * dt.itemsize, 1)
    addr, size = _pool.take(nbytes)
    buf = (ctypes.c_char * nbytes).from_address(addr)
    weakref.finalize(buf, _pool.give, addr, size)
    return np.frombuffer(buf, dtype=dt, count=count).reshape(shape)


import atexit  # noqa: E402

atexit.register(_pool.close)
