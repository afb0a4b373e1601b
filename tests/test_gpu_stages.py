"""The stage drop-ins a2-a6 (svx/stages.py: calculatePointErrors,
computePlanarThreshold, calculateColourHistogram, filterPointsByHistogram,
functions.py:212-230, :300-323) on the GPU against the reference's own outputs:
tests/golden/crops.npz (dist bits, kept / kept2 indices, bin counts) and
tests/golden/stages.json (dict items in the reference's order, the functions'
default thresholds, edge-case results and exceptions; make_stages_golden.py)."""
import json
import os
import types

import numpy as np
import pytest

from conftest import GOLDEN

pytestmark = pytest.mark.gpu
FIX = json.load(open(os.path.join(GOLDEN, "stages.json")))


@pytest.fixture(scope="module")
def mods():
    import svx
    from svx import dropin, stages
    assert svx.device_count() >= 1
    return types.SimpleNamespace(dropin=dropin, stages=stages)


@pytest.fixture(scope="module")
def crops():
    return np.load(os.path.join(GOLDEN, "crops.npz"))


def _ids(sub, points):
    pos = {id(p): i for i, p in enumerate(points)}
    return [pos[id(p)] for p in sub]


@pytest.mark.parametrize("k", [0, 1, 2])
@pytest.mark.parametrize("plain", [False, True])
def test_stages_match_reference(mods, crops, k, plain):
    S, fx = mods.stages, FIX["crops"][str(k)]
    points = mods.dropin.projectDisparityTo3d(crops[f"c{k}_disp"], 128, crops[f"c{k}_bgr"])
    if plain:   # any sequence of rows works, not only the drop-in's PointList
        points = [list(map(np.float64, p)) for p in points]
    abc = np.asarray(crops[f"c{k}_abc"], np.float64).reshape(3, 1)
    dist = S.calculatePointErrors(abc, points)
    assert list(dist.shape) == fx["dist_shape"] and dist.dtype == np.float64
    assert np.array_equal(dist.reshape(-1).view(np.uint64), crops[f"c{k}_dist"].view(np.uint64))
    kept = S.computePlanarThreshold(points, dist, 0.05)
    assert _ids(kept, points) == list(crops[f"c{k}_keep_idx"])
    hist = S.calculateColourHistogram(kept)
    assert [[key, v] for key, v in hist.items()] == fx["hist_items"]          # same keys, counts, order
    kept2 = S.filterPointsByHistogram(kept, hist, 10)
    assert _ids(kept2, points) == fx["keep2_idx"] == list(crops[f"c{k}_keep2_idx"])
    # the functions' default thresholds (0.01, 100)
    kept_d = S.computePlanarThreshold(points, dist)
    assert _ids(kept_d, points) == fx["default_keep_idx"]
    hist_d = S.calculateColourHistogram(kept_d)
    assert [[key, v] for key, v in hist_d.items()] == fx["default_hist_items"]
    assert _ids(S.filterPointsByHistogram(kept_d, hist_d), points) == fx["default_keep2_idx"]


def test_stage_edges(mods, crops):
    S, e = mods.stages, FIX["edges"]
    points = mods.dropin.projectDisparityTo3d(crops["c0_disp"], 128, crops["c0_bgr"])
    abc = np.asarray(crops["c0_abc"], np.float64)
    for call, ref in ((lambda: S.calculatePointErrors(abc.reshape(3, 1), []), e["errors_empty_points"]),
                      (lambda: S.calculatePointErrors(None, points), e["errors_none_plane"]),
                      (lambda: S.filterPointsByHistogram(points, {}, 10), e["filter_missing_key"])):
        with pytest.raises(Exception) as ei:
            call()
        assert type(ei.value).__name__ == ref["type"]
        assert [str(a) for a in ei.value.args] == ref["args"]
    assert list(S.calculatePointErrors(abc, points).shape) == e["errors_flat_plane_shape"]
    assert S.computePlanarThreshold([], np.zeros((0, 1)), 0.05) == e["threshold_empty"]
    assert S.calculateColourHistogram([]) == e["histogram_empty"]
    assert S.filterPointsByHistogram([], {}, 10) == e["filter_empty"]
    assert [[key, v] for key, v in S.calculateColourHistogram(points).items()] == e["float_rgb_hist_items"]
    bad = [list(p) for p in points[:5]]
    bad[2][3] = 12.5
    with pytest.raises(ValueError):
        S.calculateColourHistogram(bad)


def test_subset_keeps_rows_and_array(mods, crops):
    points = mods.dropin.projectDisparityTo3d(crops["c1_disp"], 128, crops["c1_bgr"])
    dist = mods.stages.calculatePointErrors(np.asarray(crops["c1_abc"]).reshape(3, 1), points)
    kept = mods.stages.computePlanarThreshold(points, dist, 0.05)
    idx = _ids(kept, points)
    assert all(kept[j] is points[i] for j, i in enumerate(idx))          # the caller's own row objects
    assert np.array_equal(kept.array(), points.array()[idx])
    points[idx[0]][0] = 123.0                                            # a write through a row view ...
    assert kept.array()[0, 0] == 123.0                                   # ... is seen by the subset's array
    kept.append(points[0])
    assert kept.array() is None                                          # a mutated list forgets it


def test_installed_chain_matches_reference(mods, crops):
    """stereovision.py:97-113 through the installed module attributes."""
    f = types.SimpleNamespace(camera_focal_length_px=399.9745178222656, stereo_camera_baseline_m=0.2090607502,
                              image_centre_w=474.5, image_centre_h=262.0)   # functions.py:15-22
    mods.dropin.install(f)
    try:
        for k in range(3):
            points = f.projectDisparityTo3d(crops[f"c{k}_disp"], 128, crops[f"c{k}_bgr"])
            abc = np.asarray(crops[f"c{k}_abc"], np.float64).reshape(3, 1)
            diffs = f.calculatePointErrors(abc, points)
            points = f.computePlanarThreshold(points, diffs, 0.05)
            hist = f.calculateColourHistogram(points)
            points = f.filterPointsByHistogram(points, hist, 10)
            pp = np.array(f.project3DPointsTo2DImagePoints(points), np.int32).reshape((-1, 1, 2))
            assert np.array_equal(pp, crops[f"c{k}_plane_points"]), k
    finally:
        mods.dropin.uninstall()
