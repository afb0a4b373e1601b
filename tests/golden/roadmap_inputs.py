"""Inputs of the imageRoadMap fixtures (make_roadmap_golden.py), shared with the
tests: (name, imgL (H, W, 3) uint8, planePoints (N, 1, 2) int32) per case."""
import json
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))


def wrap_points():
    """points with numpy's negative-index wrap and repeats (int32 (N,1,2), [x, y])"""
    p = [[-1, -1], [0, -1], [-1, 0], [5, 7], [5, 7], [1023, 543], [-1024, -544], [100, -2], [-3, 200]]
    return np.array(p, np.int32).reshape(-1, 1, 2)


def cases(digest):
    """the golden step-2 chains (their planePoints are the reference's: checked by digest), frame 0's
    chain at step 1, and the wrap set on synthetic frame 3's BGR"""
    import oracle
    meta = json.load(open(os.path.join(HERE, "digests.json")))
    for fid, m2 in meta["full_frames_step2"].items():
        disp, bgr = oracle.synth_frame(0 if fid == "0r" else int(fid))
        ref = oracle.pipeline_frame(disp, bgr, 2, abc=np.array(m2["abc"]))
        pp = ref["pts"].reshape(-1, 1, 2)
        assert digest(pp) == m2["plane_points"]          # the chain is the reference's
        yield f"step2_{fid}", bgr, pp
    disp, bgr = oracle.synth_frame(0)
    ref = oracle.pipeline_frame(disp, bgr, 1)
    yield "step1_0", bgr, ref["pts"].reshape(-1, 1, 2)
    _, bgr = oracle.synth_frame(3)
    yield "wrap", bgr, wrap_points()
