"""Host control plane for one-process-per-GPU runs, without PyTorch.

The ranks of one node (torchrun's RANK / WORLD_SIZE / LOCAL_RANK, or processes
a caller starts with those variables set) meet over plain TCP in a star: rank 0 listens
on an ephemeral port of MASTER_ADDR (default 127.0.0.1) and publishes
"host port" in a rendezvous file, the other ranks read it and connect. The
file is SVX_CTRL_FILE when set (a launcher of its own, e.g. the CPU tests, sets it), else
/tmp/svx_ctrl_<MASTER_PORT>_<parent pid>: every rank of one torchrun has the
same parent (the launcher agent), so concurrent jobs never share a file.
Single node only (the contract's --nnodes=1).

What it carries is small and rare: barriers, max/sum over ranks of a few
float64 values (timings, counts) and the 128-byte ncclUniqueId from rank 0.
The data path never touches it.
"""
import os
import socket
import struct
import tempfile
import time

import numpy as np


def rendezvous_file():
    path = os.environ.get("SVX_CTRL_FILE")
    if path:
        return path
    port = os.environ.get("MASTER_PORT", "0")
    return os.path.join(tempfile.gettempdir(), f"svx_ctrl_{port}_{os.getppid()}")


def _send(sock, data):
    sock.sendall(struct.pack("<Q", len(data)) + data)


def _recv_exact(sock, n):
    buf = bytearray()
    while len(buf) < n:
        chunk = sock.recv(n - len(buf))
        if not chunk:
            raise ConnectionError("control plane: peer closed the connection")
        buf += chunk
    return bytes(buf)


def _recv(sock):
    (n,) = struct.unpack("<Q", _recv_exact(sock, 8))
    return _recv_exact(sock, n)


class TcpControl:
    """Star-topology control plane: rank 0 holds one socket per other rank."""

    def __init__(self, rank, world, path=None, timeout=300.0):
        if not 0 <= rank < world:
            raise ValueError(f"rank {rank} outside world {world}")
        self.rank, self.world = rank, world
        self._peers = {}
        self._sock = None
        self._path = path or rendezvous_file()
        if world == 1:
            return
        deadline = time.monotonic() + timeout
        host = os.environ.get("MASTER_ADDR", "127.0.0.1")
        if rank == 0:
            srv = socket.socket(socket.AF_INET, socket.SOCK_STREAM)
            srv.setsockopt(socket.SOL_SOCKET, socket.SO_REUSEADDR, 1)
            srv.bind((host, 0))
            srv.listen(world)
            srv.settimeout(timeout)
            tmp = f"{self._path}.{os.getpid()}.tmp"
            with open(tmp, "w") as fh:
                fh.write(f"{host} {srv.getsockname()[1]}\n")
            os.replace(tmp, self._path)   # atomic: readers see the whole line or nothing
            try:
                while len(self._peers) < world - 1:
                    conn, _ = srv.accept()
                    conn.settimeout(timeout)
                    conn.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
                    (r,) = struct.unpack("<i", _recv_exact(conn, 4))
                    if not 0 < r < world or r in self._peers:
                        raise ConnectionError(f"control plane: unexpected rank {r}")
                    self._peers[r] = conn
            finally:
                srv.close()
                try:
                    os.remove(self._path)
                except OSError:
                    pass
        else:
            while True:
                try:
                    with open(self._path) as fh:
                        h, p = fh.read().split()
                    s = socket.create_connection((h, int(p)), timeout=timeout)
                    break
                except (OSError, ValueError):
                    if time.monotonic() > deadline:
                        raise TimeoutError(f"control plane: no rank 0 at {self._path}")
                    time.sleep(0.05)
            s.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
            s.sendall(struct.pack("<i", rank))
            self._sock = s

    # rank 0 gathers one message from every rank, then sends every rank the same reply
    def _exchange(self, payload, combine):
        if self.world == 1:
            return combine([payload])
        if self.rank == 0:
            msgs = [payload] + [_recv(self._peers[r]) for r in range(1, self.world)]
            out = combine(msgs)
            for r in range(1, self.world):
                _send(self._peers[r], out)
            return out
        _send(self._sock, payload)
        return _recv(self._sock)

    def barrier(self):
        self._exchange(b"", lambda msgs: b"")

    def _reduce(self, values, fn):
        a = np.ascontiguousarray(values, np.float64)
        out = self._exchange(a.tobytes(), lambda msgs: fn(
            np.stack([np.frombuffer(m, np.float64) for m in msgs]), axis=0).astype(np.float64).tobytes())
        return np.frombuffer(out, np.float64).copy()

    def max(self, values):
        return self._reduce(values, np.max)

    def sum(self, values):
        return self._reduce(values, np.sum)

    def broadcast_bytes(self, data, src=0):
        if src != 0:
            raise ValueError("control plane: broadcasts come from rank 0")
        return self._exchange(bytes(data) if self.rank == 0 else b"", lambda msgs: msgs[0])

    def close(self):
        for c in self._peers.values():
            c.close()
        self._peers = {}
        if self._sock:
            self._sock.close()
            self._sock = None
