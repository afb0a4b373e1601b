"""Parity of the disparity-stage oracle with OpenCV itself, wherever cv2 imports.

cv2 is absent from this image (and from the GPU box), so these tests skip
here; they are the harness a maintainer with OpenCV runs to pin
oracle/sgbm_oracle.c (and through it the GPU kernels, tests/test_gpu_sgbm.py)
against the library the reference calls (functions.py:26, :89-128).
"""
import numpy as np
import pytest

from oracle import sgbm as osg

cv2 = pytest.importorskip("cv2")


def test_sgbm_matches_cv2():
    sp = cv2.StereoSGBM_create(0, 128, 21)   # functions.py:26
    for fid in (0, 1):
        L, R = osg.synth_pair(fid, 272, 512)
        assert np.array_equal(osg.sgbm(L, R), sp.compute(L, R))


def test_filter_speckles_matches_cv2():
    L, R = osg.synth_pair(0, 272, 512)
    raw = osg.sgbm(L, R)
    ref = raw.copy()
    cv2.filterSpeckles(ref, 0, 4000, 123)
    assert np.array_equal(osg.filter_speckles(raw, 0, 4000, 123), ref)


def test_grey_equalize_matches_cv2():
    rng = np.random.default_rng(1)
    bgr = rng.integers(0, 256, (96, 160, 3), dtype=np.uint8)
    ref = cv2.equalizeHist(cv2.cvtColor(bgr, cv2.COLOR_BGR2GRAY))
    assert np.array_equal(osg.grey_equalize(bgr), ref)
