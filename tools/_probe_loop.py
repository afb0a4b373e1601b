"""Probe: does the two-slot FrameLoop overlap its slots? Prints per-batch stage timelines (ms since the first
submit) for a 2-slot and a 1-slot loop, and a two-stream K1 concurrency check."""
import os, sys, time
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "stereo.vision_amd"), os.path.join(REPO, "tests")]
import numpy as np
from svx import batch as sb
from svx.loop import FrameLoop, STAGES
from test_prepass_cpu import carmask
F = int(os.environ.get("PROBE_FRAMES", 4096))
mask = carmask()

def show(loop, seqs):
    for q in seqs:
        tl = loop.timeline(q)
        print(f"  batch {q}: " + "  ".join(f"{n[:4]} {tl[n][0]:8.2f}-{tl[n][1]:8.2f}" for n in STAGES), flush=True)

for slots in (2, 1):
    with FrameLoop(F, slots=slots, carmask=mask) as loop:
        for i in range(2):
            s = loop.submit(i * F)
        loop.wait(s)
        t0 = time.perf_counter()
        seqs = [loop.submit((2 + i) * F) for i in range(4)]
        t_sub = [(time.perf_counter() - t0) * 1e3]
        loop.wait(seqs[-1])
        dt = (time.perf_counter() - t0) / 4 * 1e3
        print(f"slots={slots}: {dt:.2f} ms/batch (host submit of 4 took {t_sub[0]:.1f} ms)", flush=True)
        show(loop, seqs[-slots:])

# two streams, K1 on each: concurrent?
a = sb.Batch(2048, step=1, with_bgr=False); a.synth(0)
b = sb.Batch(2048, step=1, with_bgr=False); b.synth(2048)
for x in (a, b):
    x.project(); x.project()
def t(name, fn, reps=10):
    fn(); a.sync(); b.sync()
    t0 = time.perf_counter()
    for _ in range(reps): fn()
    a.sync(); b.sync()
    print(f"{name:40s} {(time.perf_counter() - t0) / reps * 1e3:8.3f} ms", flush=True)
t("K1 a", lambda: a.project(sync=False))
t("K1 a + K1 b (two streams)", lambda: (a.project(sync=False), b.project(sync=False)))
a.close(); b.close()
