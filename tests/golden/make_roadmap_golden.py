#!/usr/bin/env python3
"""imageRoadMap fixtures from the REFERENCE's own code (stereovision.py:131-133).

CONTAINER ONLY (needs /root/reference):
    PYTHONDONTWRITEBYTECODE=1 python3 -B tests/golden/make_roadmap_golden.py

The paint is inline in performStereoVision (the rest of which needs cv2), so
this script takes the three statements from /root/reference/stereovision.py
at run time (located by their text, not copied into the repository) and
executes them unmodified with `imgL` and `planePoints` bound:

    imageRoadMap = imgL.copy(); for i in planePoints: imageRoadMap[i[0][1]][i[0][0]] = [0,255,0]

Inputs: the golden chains' int32 planePoints (stereovision.py:112-113 of the
reference-run pipeline, tests/golden/digests.json) on their synthetic BGR
frames at step 2, frame 0's chain at step 1, and a hand-made point set with
numpy's negative-index wrap (-1 = the last row / column) and repeats.
Stored in roadmap.json: digest of imageRoadMap and its count of [0, 255, 0]
pixels per case.
"""
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [HERE, REPO]
from make_golden import digest  # noqa: E402
from roadmap_inputs import cases  # noqa: E402

REF_SV = "/root/reference/stereovision.py"


def paint_statements():
    lines = open(REF_SV).read().splitlines()
    i = next(k for k, ln in enumerate(lines) if ln.strip() == "imageRoadMap = imgL.copy()")
    block = [lines[i].strip(), lines[i + 1].strip(), lines[i + 2].strip()]
    assert block[1].startswith("for i in planePoints") and block[2].startswith("imageRoadMap[")
    return i + 1, "\n".join([block[0], block[1], "    " + block[2]])


def main():
    line, code = paint_statements()
    out = {"source": f"stereovision.py:{line}-{line + 2}", "cases": {}}
    for name, bgr, pp in cases(digest):
        ns = {"imgL": bgr.copy(), "planePoints": pp}
        exec(compile(code, REF_SV, "exec"), ns)   # the reference's own statements
        img = ns["imageRoadMap"]
        assert img.shape == bgr.shape and img.dtype == np.uint8
        green = int(((img[..., 0] == 0) & (img[..., 1] == 255) & (img[..., 2] == 0)).sum())
        out["cases"][name] = {"points": int(len(pp)), "image": digest(img), "green": green,
                              "points_digest": digest(pp)}
    with open(os.path.join(HERE, "roadmap.json"), "w") as fh:
        json.dump(out, fh, indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
