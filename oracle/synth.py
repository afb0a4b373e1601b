"""ORACLE (test infrastructure only): numpy twin of the counter-based generator.

SURVEY.md §8d. Each pixel is a pure function of (frame id, y, x), so the same
frame can be regenerated on the host (here), in C (svx_oracle.c) and on the
device (the product's synth kernel) and compared byte for byte.
"""
import numpy as np

_GOLDEN = np.uint64(0x9E3779B97F4A7C15)
_M1 = np.uint64(0xBF58476D1CE4E5B9)
_M2 = np.uint64(0x94D049BB133111EB)


def mix64(z):
    z = z + _GOLDEN
    z = (z ^ (z >> np.uint64(30))) * _M1
    z = (z ^ (z >> np.uint64(27))) * _M2
    return z ^ (z >> np.uint64(31))


def frame(frame_id, H=544, W=1024):
    """(disp (H,W) u8, bgr (H,W,3) u8) for one global frame id."""
    with np.errstate(over="ignore"):
        y = np.arange(H, dtype=np.int64)[:, None]
        x = np.arange(W, dtype=np.int64)[None, :]
        idx = ((np.uint64(frame_id) * np.uint64(H) + y.astype(np.uint64)) * np.uint64(W)
               + x.astype(np.uint64))
        r = mix64(idx + np.uint64(0x5EED000000000001))
        r2 = mix64(idx + np.uint64(0x5EED000000000002))
    t = (3 * (y - 200)) // 5 + ((r >> np.uint64(8)) & np.uint64(7)).astype(np.int64) - 3
    d = np.clip(t, 0, 254) & ~1
    d = np.where((r & np.uint64(0xFF)) < np.uint64(38), 0, d).astype(np.uint8)
    lo = y >= 262
    b = np.where(lo, 110 + (r2 & np.uint64(3)), r2 & np.uint64(255))
    g = np.where(lo, 100 + ((r2 >> np.uint64(2)) & np.uint64(3)), (r2 >> np.uint64(8)) & np.uint64(255))
    rr = np.where(lo, 90 + ((r2 >> np.uint64(4)) & np.uint64(3)), (r2 >> np.uint64(16)) & np.uint64(255))
    bgr = np.stack([b, g, rr], axis=-1).astype(np.uint8)
    return d, bgr
