import sys, time
sys.path[:0] = ['/root/repo', '/root/repo/stereo.vision_amd']
from svx import batch
n = int(sys.argv[1]) if len(sys.argv) > 1 else 64
for chunk in (8, 32):
    with batch.Batch(n, 544, 1024, step=1, with_bgr=False) as b:
        b.synth_pair(0)
        b.sgbm(chunk=chunk)
        b.reset_timing()
        for _ in range(2):
            b.sgbm(chunk=chunk)
        ms, cnt = b.timing("sgbm")
        print(f"frames={n} chunk={chunk}: {ms/cnt:.2f} ms per batch, {ms/cnt/n*1000:.1f} us/frame", flush=True)
