"""Frame-loop throughput with one batch vs two batches in flight (each batch has its own stream), diagnostic.

python3 tools/loop2.py [frames] — prints ms per batch of the device frame loop (pre-pass, RANSAC, pipeline with
each frame's plane, road raster + walk) run back to back on one batch, then alternately on two."""
import json
import os
import sys
import time

R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [R, os.path.join(R, "stereo.vision_amd"), os.path.join(R, "tests")]
from svx import batch as sb   # noqa: E402
from test_prepass_cpu import carmask   # noqa: E402

frames = int(sys.argv[1]) if len(sys.argv) > 1 else 4096


def make(first):
    b = sb.Batch(frames, 544, 1024, 1, with_bgr=True, with_points=True)
    b.synth(first)
    b.set_mask(carmask())
    return b


def loop(b):
    b.prepass("previous", sync=False)
    b.ransac(seed_base=0, trials=600, sync=False)
    b.pipeline_planes(sync=False)
    b.road_raster(sync=False)
    b.nonzero(sync=False)


def loop_staged(bs):
    """the batches' stages interleaved: every batch's pre-pass and RANSAC, then every batch's pipeline and road"""
    for b in bs:
        b.prepass("previous", sync=False)
        b.ransac(seed_base=0, trials=600, sync=False)
    for b in bs:
        b.pipeline_planes(sync=False)
        b.road_raster(sync=False)
        b.nonzero(sync=False)


def timed(bs, reps, staged=False):
    def run():
        if staged:
            loop_staged(bs)
        else:
            for b in bs:
                loop(b)
    run()
    for b in bs:
        b.sync()
    t0 = time.perf_counter()
    for _ in range(reps):
        run()
    for b in bs:
        b.sync()
    return (time.perf_counter() - t0) / reps / len(bs) * 1e3


a = make(0)
one = timed([a], 4)
b2 = make(frames)
two = timed([a, b2], 4)
two_staged = timed([a, b2], 4, staged=True)
one_again = timed([a], 4)
print(json.dumps({"frames": frames, "one_batch_ms": round(one, 2), "two_batches_ms_per_batch": round(two, 2),
                  "two_batches_staged_ms_per_batch": round(two_staged, 2), "one_batch_again_ms": round(one_again, 2)}),
      flush=True)
