#!/usr/bin/env python3
"""Disparity-stage fixtures from the REFERENCE's own functions.

CONTAINER ONLY (needs /root/reference):
    PYTHONDONTWRITEBYTECODE=1 python3 -B tests/golden/make_sgbm_golden.py

The reference's disparity stage is OpenCV (absent here), wrapped in numpy code
of its own. This script runs the reference's functions unmodified with the
stub cv2 of make_golden.py, giving the stub only OpenCV's documented element
semantics, so that what it pins is the reference's OWN code around the cv2
calls:

* gammaChange (functions.py:61-67): the table is the reference's numpy
  expression; the stub's cv2.LUT is table[image] (cv2.LUT for 8-bit images).
  Stored: the tables for gamma 1.4 (preProcessImages) and 1.0.
* disparity (functions.py:104-128) after the SGBM call: the stub's
  stereoProcessor.compute returns a given int16 array, filterSpeckles is
  skipped (identity: the input is taken as already filtered), threshold is
  TOZERO at 0 (dst = src > 0 ? src : 0). What remains is the reference's
  numpy: (d / 16.).astype(uint8), the crop [0:390, 135:W] and
  (x * (256. / max_disparity)).astype(uint8). Stored: digests of its output
  for every int16 value (a 256 x 256 image of -32768..32767) and for the
  oracle's filtered SGBM (compute = computeDisparitySGBM + medianBlur 3,
  then filterSpeckles) of synthetic pairs 0 and 1, crop off/on,
  max_disparity 128 (the reference's) and 64.
StereoSGBM itself and filterSpeckles cannot run here: PARITY UNPINNED
(oracle/sgbm_oracle.c restates OpenCV's published algorithm).
"""
import json
import os
import re
import sys
import types

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [HERE, REPO]
from make_golden import digest, load_reference  # noqa: E402

from oracle import sgbm as osg  # noqa: E402


def all_int16():
    return (np.arange(65536, dtype=np.int64) - 32768).astype(np.int16).reshape(256, 256)


def oracle_inputs():
    out = {}
    for fid in (0, 1):
        L, R = osg.synth_pair(fid)
        _, _, filt = osg.disparity(L, R, with_raw=True)
        out[f"pair{fid}"] = filt
    out["all_int16"] = all_int16()
    return out


def main():
    f = load_reference()
    cv2 = f.cv2
    cv2.LUT = lambda img, table: np.asarray(table)[img]
    cv2.threshold = lambda src, thresh, maxval, typ: (thresh, np.where(src > thresh, src, 0).astype(src.dtype))
    cv2.filterSpeckles = lambda *a, **k: None
    ident = np.arange(256, dtype=np.uint8).reshape(16, 16)
    out = {"gamma": {str(g): f.gammaChange(ident, g).reshape(-1).astype(int).tolist() for g in (1.4, 1.0)}}
    pre_l, pre_r = f.preProcessImages(ident, ident[::-1].copy())
    assert (pre_l == np.asarray(out["gamma"]["1.4"], np.uint8).reshape(16, 16)).all()
    scaled = {}
    for name, arr in oracle_inputs().items():
        f.stereoProcessor = types.SimpleNamespace(compute=lambda L, R, a=arr: a.copy())
        rec = {"in": digest(arr), "shape": list(arr.shape)}
        for md in (128, 64):
            for crop in (False, True):
                r = f.disparity(None, None, md, crop)
                rec[f"md{md}_crop{int(crop)}"] = {"digest": digest(r), "shape": list(r.shape)}
        scaled[name] = rec
    out["scaled"] = scaled
    text = json.dumps(out, indent=1, separators=(",", ": "))
    # integer lists (the gamma tables) on one line each
    text = re.sub(r"\[\s*(-?\d+(?:,\s*-?\d+)*)\s*\]", lambda m: "[" + re.sub(r"\s+", "", m.group(1)) + "]", text)
    with open(os.path.join(HERE, "sgbm.json"), "w") as fh:
        fh.write(text)
    print("wrote sgbm.json")


if __name__ == "__main__":
    main()
