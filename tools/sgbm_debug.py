"""Diagnostic: GPU filterSpeckles vs the oracle on the full-frame SGBM output."""
import sys, numpy as np
sys.path[:0] = ['/root/repo', '/root/repo/stereo.vision_amd']
from svx import disparity as sd
from oracle import sgbm as osg
L, R = osg.synth_pair(0)
raw = osg.sgbm(L, R)
ref = osg.filter_speckles(raw, 0, 4000, 123)
for trial in range(3):
    g = raw.copy()
    sd.filterSpeckles(g, 0, 4000, 123)
    bad = np.argwhere(g != ref)
    print('trial', trial, 'mismatches', len(bad), 'gpu zeroed', int(((g == 0) & (raw != 0)).sum()),
          'ref zeroed', int(((ref == 0) & (raw != 0)).sum()), flush=True)
    if len(bad):
        print(bad[:10].tolist(), [(int(raw[y, x]), int(g[y, x]), int(ref[y, x])) for y, x in bad[:10]])
np.save('gpurun_out/raw0.npy', raw)
rng = np.random.default_rng(3)
img = (rng.integers(-2, 6, (544, 1024)) * 7).astype(np.int16)
g = img.copy(); sd.filterSpeckles(g, 0, 4000, 123)
print('random 544x1024 mismatches', int((g != osg.filter_speckles(img, 0, 4000, 123)).sum()))
