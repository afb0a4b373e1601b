"""svx — MI355X-native disparity -> 3D point-cloud hot path of thien/stereo.vision.

Layers (bottom-up):
  K    hand-written gfx950 HIP kernels        csrc/kernels/*.hip
  R    C++ runtime (device, streams, buffers) csrc/runtime.hip, csrc/comm.hip (RCCL)
  ABI  extern "C" libsvx.so                   include/svx.h
  P    ctypes binding + drop-in + batch API   svx/_abi.py, svx/dropin.py, svx/batch.py
       multi-GPU driver (one process per GPU) svx/dist.py
"""
from ._abi import SvxError, device_count, lib  # noqa: F401

__version__ = "0.1.0"


def version():
    return lib().sv_version().decode()
