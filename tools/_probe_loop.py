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

ONLY = os.environ.get("PROBE_ONLY")   # e.g. "caller2": that configuration alone, nothing after it
for source, slots in (("caller", 2), ("caller", 1), ("synth", 2), ("caller", 3), ("synth", 3)):
    if ONLY and f"{source}{slots}" not in ONLY.split(","):
        continue
    with FrameLoop(F, slots=slots, source=source, carmask=mask) as loop:
        NB = int(os.environ.get("PROBE_BATCHES", 6))   # batches submitted: 2 warm-up, NB - 2 timed
        for i in range(NB):
            if i == 2:
                loop.wait(s)
                # PROBE_ABLATE (diagnostic build): SVX_RANSAC_ABLATE for the timed batches only, so their evaluation
                # reads the first batches' (valid) scratch
                if os.environ.get("PROBE_ABLATE"):
                    os.environ["SVX_RANSAC_ABLATE"] = os.environ["PROBE_ABLATE"]
                t0 = time.perf_counter()
            if source == "caller" and i < slots:
                loop.acquire().synth(i * F)
            s = loop.submit(i * F)
        loop.wait(s)
        dt = (time.perf_counter() - t0) / (NB - 2) * 1e3
        os.environ.pop("SVX_RANSAC_ABLATE", None) if os.environ.get("PROBE_ABLATE") else None
        print(f"source={source} slots={slots}: {dt:.2f} ms/batch", flush=True)
        show(loop, range(s - slots + 1, s + 1))

if ONLY and not os.environ.get("PROBE_RANSAC"):
    sys.exit(0)
# the batched RANSAC alone (maskpoints + draw + eval), 4096 carmask frames
with sb.Batch(F, step=1, with_bgr=True, with_points=True) as rb:
    rb.synth(0); rb.set_mask(mask); rb.prepass("previous")
    rb.ransac(seed_base=0, trials=600)
    t0 = time.perf_counter()
    for _ in range(5):
        rb.ransac(seed_base=0, trials=600, sync=False)
    rb.sync()
    print(f"ransac alone: {(time.perf_counter() - t0) / 5 * 1e3:.3f} ms", flush=True)
if ONLY:
    sys.exit(0)

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
