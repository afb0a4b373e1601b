"""Multi-GPU driver: one process per GPU, frames sharded by global id.

SURVEY §8e: frames are independent (every reduction — hue histogram, counts —
is per frame), so a B-frame job is split into contiguous frame-id ranges, one
per rank, with no data-path collective. The only device-data exchange is the
RCCL broadcast of the plane coefficients from rank 0 over xGMI (the plane is
produced once — by RANSAC in the reference, stereovision.py:94 — and every
rank filters against it). Host control (barriers, max-over-ranks timing, the
RCCL unique-id hand-off) goes over a gloo process group.

Launch: ``torchrun --nproc-per-node N ...`` (RANK / WORLD_SIZE / LOCAL_RANK /
MASTER_ADDR / MASTER_PORT from the environment).
"""
import ctypes
import os

import numpy as np

from . import _abi


def env_topology():
    """(rank, world, local_rank) from the torchrun environment (defaults: 1 process)."""
    return (int(os.environ.get("RANK", 0)), int(os.environ.get("WORLD_SIZE", 1)),
            int(os.environ.get("LOCAL_RANK", 0)))


def shard(total, world, rank):
    """Contiguous [first, first+count) slice of `total` frames for `rank`."""
    base, extra = divmod(total, world)
    count = base + (1 if rank < extra else 0)
    first = rank * base + min(rank, extra)
    return first, count


class Control:
    """Host control plane (gloo). world == 1 needs no process group at all."""

    def __init__(self, rank=None, world=None):
        r, w, _ = env_topology()
        self.rank = r if rank is None else rank
        self.world = w if world is None else world
        self._dist = None
        if self.world > 1:
            import torch.distributed as dist
            if not dist.is_initialized():
                dist.init_process_group("gloo", rank=self.rank, world_size=self.world)
            self._dist = dist

    def barrier(self):
        if self._dist:
            self._dist.barrier()

    def _reduce(self, values, op):
        if not self._dist:
            return np.asarray(values, np.float64)
        import torch
        t = torch.tensor(np.asarray(values, np.float64))
        self._dist.all_reduce(t, op=op)
        return t.numpy()

    def max(self, values):
        import torch.distributed as dist  # noqa: F401 (op enum)
        return self._reduce(values, self._dist.ReduceOp.MAX if self._dist else None)

    def sum(self, values):
        return self._reduce(values, self._dist.ReduceOp.SUM if self._dist else None)

    def broadcast_bytes(self, data, src=0):
        """Broadcast a bytes object of fixed length from `src`."""
        if not self._dist:
            return bytes(data)
        import torch
        n = len(data)
        t = torch.tensor(np.frombuffer(bytes(data), np.uint8).copy())
        self._dist.broadcast(t, src=src)
        return bytes(t.numpy().tobytes()[:n])

    def close(self):
        if self._dist and self._dist.is_initialized():
            self._dist.destroy_process_group()


class RcclComm:
    """RCCL communicator over the node's GPUs (sv_comm_* in libsvx)."""

    def __init__(self, ctrl, device):
        uid = (ctypes.c_uint8 * _abi.SV_UNIQUE_ID_BYTES)()
        if ctrl.rank == 0:
            _abi.call("sv_comm_unique_id", ctypes.cast(uid, ctypes.c_void_p))
        data = ctrl.broadcast_bytes(bytes(uid), src=0)
        uid = (ctypes.c_uint8 * _abi.SV_UNIQUE_ID_BYTES).from_buffer_copy(data)
        h = ctypes.c_void_p()
        _abi.call("sv_comm_init", ctrl.world, ctrl.rank, ctypes.cast(uid, ctypes.c_void_p), device,
                  ctypes.byref(h))
        self._h = h

    def broadcast_plane(self, plane, root=0):
        pl = _abi.Plane(*plane)
        _abi.call("sv_comm_broadcast_plane", self._h, ctypes.byref(pl), root)
        return (pl.a, pl.b, pl.c)

    def allreduce_i64(self, values):
        a = np.ascontiguousarray(values, np.int64).copy()
        _abi.call("sv_comm_allreduce_i64", self._h, _abi.ptr(a), a.size)
        return a

    def close(self):
        if self._h:
            _abi.call("sv_comm_destroy", self._h)
            self._h = None
