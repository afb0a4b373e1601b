#!/usr/bin/env python3
"""Generate tests/golden/frame_digests.npz: per-frame digests of the synthetic
frames at BASELINE.json's full sizes, from the pinned C oracle (oracle/svx_oracle.c
svo_frame_digest; the oracle is itself pinned to the reference's own outputs by
tests/test_oracle_golden.py).

  step1: frames 0..32767 at step 1 — configs[2]/[3] (4096 frames on one GPU) and
         configs[4] (32,768 frames sharded over 8 GPUs by global frame id)
  step2: frames 0..4095 at step 2 (the reference's hard-coded step)

Each row: n_valid, n_kept, n_kept2 (the counts of stereovision.py:84-113 with the
SURVEY §8d plane and thresholds 0.05 / 10) and three 64-bit hashes (disparity,
hue histogram, surviving points in order with their int32 back-projection); see
the definitions above svo_frame_digest. The GPU tests and bench.py compare the
device's own digests of every frame with these rows.

usage: python tests/golden/make_frame_digests.py   (about 2 minutes on 8 cores)
"""
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

import oracle  # noqa: E402


def main():
    t0 = time.time()
    step1 = oracle.frame_digests(0, 32768, step=1)
    print(f"step 1: {len(step1)} frames, {time.time() - t0:.1f} s", flush=True)
    step2 = oracle.frame_digests(0, 4096, step=2)
    print(f"step 2: {len(step2)} frames, {time.time() - t0:.1f} s", flush=True)
    np.savez_compressed(os.path.join(HERE, "frame_digests.npz"), step1=step1, step2=step2)


if __name__ == "__main__":
    main()
