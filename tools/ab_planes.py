#!/usr/bin/env python3
"""A/B helper: ms per call of the per-frame-plane pipeline (after batched RANSAC)
and of the tiled single-plane pipeline on 4096 synthetic frames (one process)."""
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "stereo.vision_amd")]
from svx import batch as sb  # noqa: E402

b = sb.Batch(4096, step=1, with_bgr=True, with_points=True)
b.synth(0)
mask = __import__("numpy").zeros((544, 1024), __import__("numpy").uint8)
mask[544 // 3:, 64:1024 - 64] = 255
b.set_mask(mask)
b.prepass("previous")
b.ransac(seed_base=0, trials=600)
for name, fn in (("planes", lambda: b.pipeline_planes(sync=False)),
                 ("tiled", lambda: (b.pipeline_mode("tiled"), b.pipeline(sync=False)))):
    fn()
    b.sync()
    t0 = time.perf_counter()
    for _ in range(5):
        fn()
    b.sync()
    print(name, "ms", round((time.perf_counter() - t0) / 5 * 1e3, 3), "kept", int(b.read_counts()[:, 2].sum()),
          flush=True)
b.close()
