import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(REPO, "stereo.vision_amd")
for p in (REPO, PKG):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN = os.path.join(REPO, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs on the GPU box)")
    config.addinivalue_line("markers", "slow: long CPU test")


@pytest.fixture(scope="session")
def golden():
    import json

    import numpy as np

    class G:
        sparse = np.load(os.path.join(GOLDEN, "sparse.npz"))
        crops = np.load(os.path.join(GOLDEN, "crops.npz"))
        hue = np.load(os.path.join(GOLDEN, "hue_sample.npz"))
        deltas = np.load(os.path.join(GOLDEN, "deltas.npz"))
        with open(os.path.join(GOLDEN, "digests.json")) as fh:
            meta = json.load(fh)
    return G


def sparse_frame(golden, k):
    """Rebuild sparse fixture frame k: zeros + listed pixels, synthetic bgr + overrides."""
    import oracle

    pix = golden.sparse[f"f{k}_pix"]
    disp = __import__("numpy").zeros((544, 1024), "uint8")
    disp[pix[:, 0], pix[:, 1]] = pix[:, 2]
    _, bgr = oracle.synth_frame(int(golden.sparse[f"f{k}_frame_id"]))
    bgr[pix[:, 0], pix[:, 1]] = golden.sparse[f"f{k}_pix_bgr"]
    return disp, bgr
