#!/usr/bin/env python3
"""Fixtures for the a2-a6 stage drop-ins (functions.py:212-230, :300-323),
made by running the REFERENCE's own functions. CONTAINER ONLY (needs
/root/reference); run as

    PYTHONDONTWRITEBYTECODE=1 python3 -B tests/golden/make_stages_golden.py

Inputs are the crops already in crops.npz (disp, bgr, abc). Saved (data only)
to stages.json:
* per crop: calculateColourHistogram's items in the dict's own order (the
  first-occurrence order the reference builds), the shape of
  calculatePointErrors' result, and the same four stages with the functions'
  default thresholds (computePlanarThreshold 0.01, filterPointsByHistogram 100);
* edge cases: the exception type (and KeyError key) the reference raises for
  empty points, a missing plane, a histogram without a point's key; the
  result for empty lists and for a (3,) plane.
"""
import json
import os
import sys

import numpy as np

OUT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, OUT)
from make_golden import load_reference  # noqa: E402


def ids_in(sub, points):
    pos = {id(p): i for i, p in enumerate(points)}
    return [pos[id(p)] for p in sub]


def raised(fn):
    try:
        fn()
    except Exception as e:   # noqa: BLE001  (recording the reference's behaviour)
        return {"type": type(e).__name__, "args": [str(a) for a in e.args]}
    return None


def main():
    F = load_reference()
    crops = np.load(os.path.join(OUT, "crops.npz"))
    out = {"crops": {}, "edges": {}}
    for k in range(3):
        disp, bgr, abc = crops[f"c{k}_disp"], crops[f"c{k}_bgr"], crops[f"c{k}_abc"]
        points = F.projectDisparityTo3d(disp, 128, bgr)
        abc_col = np.asarray(abc, np.float64).reshape(3, 1)
        dist = F.calculatePointErrors(abc_col, points)
        kept = F.computePlanarThreshold(points, dist, 0.05)
        hist = F.calculateColourHistogram(kept)
        kept2 = F.filterPointsByHistogram(kept, hist, 10)
        # the functions' own default thresholds
        kept_d = F.computePlanarThreshold(points, dist)
        hist_d = F.calculateColourHistogram(kept_d)
        kept2_d = F.filterPointsByHistogram(kept_d, hist_d)
        out["crops"][str(k)] = {
            "dist_shape": list(dist.shape),
            "hist_items": [[key, int(v)] for key, v in hist.items()],
            "keep2_idx": ids_in(kept2, points),
            "default_keep_idx": ids_in(kept_d, points),
            "default_hist_items": [[key, int(v)] for key, v in hist_d.items()],
            "default_keep2_idx": ids_in(kept2_d, points),
        }
        print("crop", k, len(points), len(kept), len(hist), len(kept2), len(kept_d), len(kept2_d))
    disp, bgr, abc = crops["c0_disp"], crops["c0_bgr"], crops["c0_abc"]
    points = F.projectDisparityTo3d(disp, 128, bgr)
    abc_col = np.asarray(abc, np.float64).reshape(3, 1)
    e = out["edges"]
    e["errors_empty_points"] = raised(lambda: F.calculatePointErrors(abc_col, []))
    e["errors_none_plane"] = raised(lambda: F.calculatePointErrors(None, points))
    e["errors_flat_plane_shape"] = list(F.calculatePointErrors(np.asarray(abc, np.float64), points).shape)
    e["threshold_empty"] = F.computePlanarThreshold([], np.zeros((0, 1)), 0.05)
    e["histogram_empty"] = F.calculateColourHistogram([])
    e["filter_missing_key"] = raised(lambda: F.filterPointsByHistogram(points, {}, 10))
    e["filter_empty"] = F.filterPointsByHistogram([], {}, 10)
    # rows of an (N, 6) float64 array (RGB as float64): same keys as numpy uint8 scalars
    arr = np.array([list(p) for p in points], np.float64)
    rows = list(arr)
    e["float_rgb_hist_items"] = [[key, int(v)] for key, v in F.calculateColourHistogram(rows).items()]
    with open(os.path.join(OUT, "stages.json"), "w") as fh:
        json.dump(out, fh, separators=(",", ":"))
    print("wrote stages.json", os.path.getsize(os.path.join(OUT, "stages.json")), "bytes")


if __name__ == "__main__":
    main()
