"""RANSAC drop-in (functions.py:278-298) on the GPU against the reference-run
fixtures (plane bits, same-object return, random state afterwards) and the
oracle's per-trial errors."""
import json
import os
import random
import types

import numpy as np
import pytest

from conftest import GOLDEN
from oracle import ransac as oransac
from test_ransac_cpu import FIX, bits, cases, state_digest  # noqa: F401  (fixture)

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def svx_mod():
    import svx
    from svx import dropin, ransac
    assert svx.device_count() >= 1
    return types.SimpleNamespace(svx=svx, dropin=dropin, ransac=ransac)


def test_ransac_matches_reference(svx_mod, cases):   # noqa: F811
    saved = random.getstate()
    try:
        for key, ref in FIX.items():
            name, seed = key.split("/")
            random.seed(int(seed))
            normal, abc = svx_mod.ransac.RANSAC(list(cases[name]), ref["trials"])
            assert (None if abc is None else bits(abc)) == ref["abc_bits"], key
            if abc is not None:
                assert normal is abc and abc.shape == (3, 1)
            assert state_digest() == ref["state_after"], key
    finally:
        random.setstate(saved)


def test_per_trial_errors_match_oracle(svx_mod, cases):   # noqa: F811
    pts = cases["frame0"]
    st = random.Random(99).getstate()
    g = svx_mod.ransac.trials_gpu(list(pts), 300, state=st)
    r = random.Random(99)
    _, recs = oransac.ransac(pts, 300, rng=r)
    assert g["state_after"] == r.getstate()
    assert len(recs) == len(g["err"]) == 300
    for t, rec in enumerate(recs):
        assert list(g["sidx"][t]) == rec["idx"] and tuple(g["tri"][t]) == rec["tri"]
        if rec["err"] is None:
            assert g["flag"][t] != 0
        elif g["flag"][t] == 0:
            assert abs(g["err"][t] - rec["err"]) <= 1e-9 * rec["err"]
            ref = rec["abc"].reshape(3)
            np.testing.assert_allclose(g["abc"][t], ref, rtol=0, atol=1e-9 * np.linalg.norm(ref))


def test_ransac_installed_and_degenerate(svx_mod, cases):   # noqa: F811
    f = types.SimpleNamespace(RANSAC=None)
    svx_mod.dropin.install(f)
    try:
        assert f.RANSAC is svx_mod.ransac.RANSAC
        st = random.getstate()
        assert f.RANSAC(np.zeros((700, 3)), 5) == (None, None)       # ndarray: random.sample raises (TypeError)
        assert f.RANSAC(list(np.zeros((10, 3))), 5) == (None, None)  # fewer than 600 points
        assert random.getstate() == st
    finally:
        svx_mod.dropin.uninstall()
