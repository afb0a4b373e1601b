"""Deterministic point sets for the RANSAC fixtures (functions.py:240-298),
shared by make_ransac_golden.py and the tests (only outputs are stored)."""
import numpy as np


def maskpoints(oracle, carmask, frame_id):
    """stereovision.py:85: projectDisparityTo3d(maskDisparity(disparity), 128)
    on a synthetic frame (step 2, the reference's grid), as an (N, 3) array."""
    disp, _ = oracle.synth_frame(frame_id)
    xyz, _ = oracle.project(oracle.mask_disparity(disp, carmask), None, 2)
    return xyz


def degenerate_collinear():
    """650 points on one line (most triples collinear: retries) + 50 generic."""
    rng = np.random.default_rng(21)
    t = rng.integers(1, 400, 650).astype(np.float64)
    line = np.stack([t * 0.25, t * -0.5, 3.0 + t], axis=1)
    other = rng.normal(0, 5, (50, 3)) + np.array([0.0, 2.0, 20.0])
    pts = np.concatenate([line, other])
    return pts[rng.permutation(len(pts))]


def degenerate_singular():
    """Points with Z == 0 (any triple of them: singular 3x3, LinAlgError) + some off-plane."""
    rng = np.random.default_rng(22)
    flat = np.concatenate([rng.normal(0, 10, (640, 2)), np.zeros((640, 1))], axis=1)
    other = rng.normal(0, 5, (60, 3)) + np.array([0.0, 2.0, 20.0])
    pts = np.concatenate([flat, other])
    return pts[rng.permutation(len(pts))]


CASES = {   # name -> (trials, seeds)
    "frame0": (600, (0, 1, 12345)),
    "frame1": (100, (7,)),
    "frame0_n2000": (200, (3,)),
    "frame0_n599": (50, (4,)),
    "frame0_rgb": (60, (5,)),
    "collinear": (50, (6,)),
    "singular": (50, (8,)),
}


def case_points(name, oracle, carmask):
    if name.startswith("frame0"):
        p = maskpoints(oracle, carmask, 0)
        if name == "frame0_n2000":
            return p[:2000]
        if name == "frame0_n599":
            return p[:599]
        if name == "frame0_rgb":
            rgb = (np.arange(len(p) * 3).reshape(-1, 3) % 251).astype(np.float64)
            return np.concatenate([p, rgb], axis=1)
        return p
    if name == "frame1":
        return maskpoints(oracle, carmask, 1)
    if name == "collinear":
        return degenerate_collinear()
    return degenerate_singular()
