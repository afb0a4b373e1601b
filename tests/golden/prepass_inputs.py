"""Deterministic inputs for the pre-pass / rasterisation fixtures (shared by
make_prepass_golden.py and the tests, so only outputs are stored)."""
import numpy as np


def fill_mean_inputs(synth_frame):
    """Frames for fillAltDisparity (functions.py:150-162): a synthetic frame with
    zeroed rows, all-zero rows, rows of only 0/1, rows of 1s; a random frame
    with many values < 2; a small odd-width frame (row padding)."""
    d0, _ = synth_frame(3)
    d0 = d0.copy()
    d0[10] = 0                      # no non-zero value: mean is nan -> 0
    d0[11, ::2] = 1                 # only 0/1: mean of the 1s
    d0[12] = 1                      # all 1: mean 1, every pixel < 2 -> 1
    d0[300:310, 500:900] = 0
    rng = np.random.default_rng(7)
    d1 = rng.integers(0, 256, (544, 1024)).astype(np.uint8)
    d1[rng.random((544, 1024)) < 0.3] = 0
    d1[rng.random((544, 1024)) < 0.1] = 1
    d2 = rng.integers(0, 4, (7, 13)).astype(np.uint8)
    return [d0, d1, d2]


def fill_prev_inputs():
    """(disparity, previous) pairs for fillDisparity (functions.py:141-148)."""
    rng = np.random.default_rng(8)
    out = []
    for H, W in ((544, 1024), (5, 11)):
        d = rng.integers(0, 256, (H, W)).astype(np.uint8)
        d[rng.random((H, W)) < 0.4] = rng.integers(0, 3, 1)[0]
        p = rng.integers(0, 256, (H, W)).astype(np.uint8)
        out.append((d, p))
    return out
