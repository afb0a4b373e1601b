#!/usr/bin/env python3
"""Pre-pass and road-raster fixtures from the REFERENCE's own functions.

CONTAINER ONLY (needs /root/reference):
    PYTHONDONTWRITEBYTECODE=1 python3 -B tests/golden/make_prepass_golden.py

* carmask.npz  — the nonzero set of functions.py:35's carmask
                 (bitwise_and(car_front_mask, car_front_mask, mask=view_range)),
                 read from the reference's masks/*.png with PIL. cv2 is absent;
                 its grey conversion cannot zero any pixel of these masks
                 (car_front_mask is grey already, view_range's smallest channel
                 is 85), so the nonzero set does not depend on it.
* prepass.json — digests of functions.fillAltDisparity (pure numpy, runs
                 unmodified) on the inputs of prepass_inputs.py, and of
                 functions.generatePointsAsImage (functions.py:339-344, with its
                 module-level blackImg supplied as the all-zero grey image that
                 masks/black.png decodes to) on the golden step-2 chains.
fillDisparity / maskDisparity call cv2 (absent): their tests restate OpenCV's
documented semantics (threshold BINARY, bitwise_not/and with mask, saturating
add) and have no reference-run fixture.
"""
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [HERE, REPO]
from make_golden import digest, load_reference  # noqa: E402
import prepass_inputs  # noqa: E402

import oracle  # noqa: E402


def main():
    from PIL import Image
    f = load_reference()
    m = lambda n: np.array(Image.open(os.path.join("/root/reference/masks", n + ".png")))  # noqa: E731
    car, view, black = m("car_front_mask"), m("view_range"), m("black")
    assert (car[..., 0] == car[..., 1]).all() and (car[..., 1] == car[..., 2]).all()
    assert not black[..., :3].any()
    nz = (car[..., 0] > 0) & (view[..., :3].max(axis=2) > 0)
    np.savez_compressed(os.path.join(HERE, "carmask.npz"), bits=np.packbits(nz), shape=np.array(nz.shape))
    out = {"carmask_nonzero": int(nz.sum()), "carmask_digest": digest(nz.astype(np.uint8))}
    fm = []
    for d in prepass_inputs.fill_mean_inputs(oracle.synth_frame):
        r = f.fillAltDisparity(d.copy())
        fm.append({"shape": list(d.shape), "in": digest(d), "out": digest(r)})
    out["fill_mean"] = fm
    f.blackImg = np.zeros((544, 1024), np.uint8)
    raster = {}
    meta = json.load(open(os.path.join(HERE, "digests.json")))
    for fid, m2 in meta["full_frames_step2"].items():
        disp, bgr = oracle.synth_frame(0 if fid == "0r" else int(fid))
        ref = oracle.pipeline_frame(disp, bgr, 2, abc=np.array(m2["abc"]))
        pp = ref["pts"].reshape(-1, 1, 2)
        assert digest(pp) == m2["plane_points"]          # the chain is the reference's
        img = f.generatePointsAsImage(pp)
        raster[fid] = {"image": digest(img), "nonzero": int((img != 0).sum())}
    out["road_raster_step2"] = raster
    with open(os.path.join(HERE, "prepass.json"), "w") as fh:
        json.dump(out, fh, indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
