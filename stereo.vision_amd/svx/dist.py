"""Multi-GPU driver: frames sharded by global id over the GPUs of one node.

SURVEY §8e: frames are independent (every reduction — hue histogram, counts —
is per frame), so a B-frame job is split into contiguous frame-id ranges, one
per GPU, with no data-path collective. The only device-data exchange is the
RCCL broadcast of the plane coefficients from the root over xGMI (the plane is
produced once — by RANSAC in the reference, stereovision.py:94 — and every
GPU filters against it), written into device memory where the pipeline reads
it (sv_comm_broadcast_plane_dev + sv_batch_pipeline_dev): no host copy on the
receivers, no host sync per step.

Two ways to run N GPUs:
  * one process per GPU (``torchrun --nproc-per-node N``):
    RANK / WORLD_SIZE / LOCAL_RANK from the environment, host control over
    svx.control.TcpControl (no PyTorch), RcclComm per rank;
  * one process driving all N: MultiComm (ncclCommInitAll), one
    sv_batch per device, the broadcast of all devices in one RCCL group.
"""
import ctypes
import os

import numpy as np

from . import _abi
from .control import TcpControl


def env_topology():
    """(rank, world, local_rank) from the launcher's environment (defaults: 1 process)."""
    return (int(os.environ.get("RANK", 0)), int(os.environ.get("WORLD_SIZE", 1)),
            int(os.environ.get("LOCAL_RANK", 0)))


def shard(total, world, rank):
    """Contiguous [first, first+count) slice of `total` frames for `rank`."""
    base, extra = divmod(total, world)
    count = base + (1 if rank < extra else 0)
    first = rank * base + min(rank, extra)
    return first, count


class Control:
    """Host control plane of one rank: TCP (svx.control) by default; SVX_CONTROL=gloo
    uses a torch.distributed gloo group instead (same operations). World 1 needs
    neither."""

    def __init__(self, rank=None, world=None):
        r, w, _ = env_topology()
        self.rank = r if rank is None else rank
        self.world = w if world is None else world
        self._dist = None
        self._tcp = None
        if self.world > 1:
            if os.environ.get("SVX_CONTROL", "tcp") == "gloo":
                import torch.distributed as dist
                if not dist.is_initialized():
                    dist.init_process_group("gloo", rank=self.rank, world_size=self.world)
                self._dist = dist
            else:
                self._tcp = TcpControl(self.rank, self.world)

    def barrier(self):
        if self._tcp:
            self._tcp.barrier()
        elif self._dist:
            self._dist.barrier()

    def _reduce(self, values, op):
        if self._tcp:
            return self._tcp.max(values) if op == "max" else self._tcp.sum(values)
        if not self._dist:
            return np.asarray(values, np.float64)
        import torch
        t = torch.tensor(np.asarray(values, np.float64))
        self._dist.all_reduce(t, op=self._dist.ReduceOp.MAX if op == "max" else self._dist.ReduceOp.SUM)
        return t.numpy()

    def max(self, values):
        return self._reduce(values, "max")

    def sum(self, values):
        return self._reduce(values, "sum")

    def broadcast_bytes(self, data, src=0):
        """Broadcast a bytes object of fixed length from `src`."""
        if self._tcp:
            return self._tcp.broadcast_bytes(data, src)
        if not self._dist:
            return bytes(data)
        import torch
        n = len(data)
        t = torch.tensor(np.frombuffer(bytes(data), np.uint8).copy())
        self._dist.broadcast(t, src=src)
        return bytes(t.numpy().tobytes()[:n])

    def close(self):
        if self._tcp:
            self._tcp.close()
            self._tcp = None
        if self._dist and self._dist.is_initialized():
            self._dist.destroy_process_group()
        self._dist = None


class RcclComm:
    """RCCL communicator of one rank (sv_comm_* in libsvx), one process per GPU."""

    def __init__(self, ctrl, device):
        """Every rank agrees on the outcome of each setup step (ctrl.sum of a failure flag) before the next
        collective one, so a failure on some ranks raises SvxError on all of them instead of leaving the others
        waiting in a broadcast or in the collective init. (A rank that fails INSIDE ncclCommInitRank while the
        others wait in it cannot be caught from here; the device check before it makes that unlikely.)"""
        self._h = None
        self.rank = ctrl.rank
        uid = (ctypes.c_uint8 * _abi.SV_UNIQUE_ID_BYTES)()
        err = None
        try:
            _abi.call("sv_init", device)   # the device is there and selectable, before any collective step
            if ctrl.rank == 0:
                _abi.call("sv_comm_unique_id", ctypes.cast(uid, ctypes.c_void_p))
        except _abi.SvxError as e:
            err = e
        self._agree(ctrl, err, "device check / ncclGetUniqueId")
        data = ctrl.broadcast_bytes(bytes(uid), src=0)
        uid = (ctypes.c_uint8 * _abi.SV_UNIQUE_ID_BYTES).from_buffer_copy(data)
        h = ctypes.c_void_p()
        try:
            _abi.call("sv_comm_init", ctrl.world, ctrl.rank, ctypes.cast(uid, ctypes.c_void_p), device,
                      ctypes.byref(h))
        except _abi.SvxError as e:
            err = e
        if err is None:
            self._h = h
        try:
            self._agree(ctrl, err, "ncclCommInitRank")
        except _abi.SvxError:
            self.close()
            raise

    @staticmethod
    def _agree(ctrl, err, step):
        failed = int(ctrl.sum([0.0 if err is None else 1.0])[0])
        if failed:
            raise _abi.SvxError(f"RCCL {step} failed on {failed} of {ctrl.world} rank(s)"
                                + (f"; this rank: {err}" if err is not None else ""))

    def broadcast_plane(self, plane, root=0):
        """Host round trip (reporting/tests)."""
        pl = _abi.Plane(*plane)
        _abi.call("sv_comm_broadcast_plane", self._h, ctypes.byref(pl), root)
        return (pl.a, pl.b, pl.c)

    def broadcast_plane_dev(self, batch, plane, root=0):
        """The root's plane into this rank's device memory on `batch`'s stream;
        returns the device pointer for batch.pipeline_dev (no host sync)."""
        pl = _abi.Plane(*plane) if self.rank == root else None
        out = ctypes.c_void_p()
        _abi.call("sv_comm_broadcast_plane_dev", self._h, batch._h, ctypes.byref(pl) if pl else None, root,
                  ctypes.byref(out))
        return out.value

    def allreduce_i64(self, values):
        a = np.ascontiguousarray(values, np.int64).copy()
        _abi.call("sv_comm_allreduce_i64", self._h, _abi.ptr(a), a.size)
        return a

    def close(self):
        if self._h:
            _abi.call("sv_comm_destroy", self._h)
            self._h = None


class MultiComm:
    """One process driving `devices` (ncclCommInitAll; rank i on devices[i])."""

    def __init__(self, devices):
        self.devices = list(devices)
        n = len(self.devices)
        devs = (ctypes.c_int * n)(*self.devices)
        self._hs = (ctypes.c_void_p * n)()
        _abi.call("sv_comm_init_all", n, ctypes.cast(devs, ctypes.c_void_p), ctypes.cast(self._hs, ctypes.c_void_p))

    def pipeline(self, batches, plane, root=0, point_thr=0.05, hist_thr=10, camera=None, sync=False):
        """sv_multi_pipeline: grouped broadcast of `plane` from device `root`, then
        every batch's pipeline with its device's copy."""
        from .batch import CAMERA
        n = len(self.devices)
        if len(batches) != n:
            raise ValueError(f"{len(batches)} batches for {n} devices")
        hs = (ctypes.c_void_p * n)(*[b._h.value for b in batches])
        cam = camera or CAMERA
        _abi.call("sv_multi_pipeline", n, ctypes.cast(self._hs, ctypes.c_void_p), ctypes.cast(hs, ctypes.c_void_p),
                  ctypes.byref(cam), ctypes.byref(_abi.Plane(*plane)), root, float(point_thr), int(hist_thr),
                  int(sync))

    def close(self):
        if self._hs is not None:
            for h in self._hs:
                if h:
                    _abi.call("sv_comm_destroy", ctypes.c_void_p(h))
            self._hs = None
