"""Pin the oracle (C restatement + nested-loop port) to the reference's own outputs.

Fixtures in tests/golden/ were produced by running the reference functions
(functions.py / stereovision.py, unmodified) — see tests/golden/make_golden.py.
CPU only.
"""
import numpy as np
import pytest

import oracle
from oracle import cpu_loop
from oracle import synth as osynth
from conftest import sparse_frame


def _chain_c(disp, bgr, abc, step=2):
    xyz, rgb = oracle.project(disp, bgr, step)
    dist = oracle.point_errors(xyz, abc) if len(xyz) else np.zeros(0)
    r = oracle.pipeline_frame(disp, bgr, step, abc=abc)
    return xyz, rgb, dist, r


def _check_chain(prefix, store, disp, bgr, abc):
    xyz, rgb, dist, r = _chain_c(disp, bgr, abc)
    ref_xyz = store[f"{prefix}_xyz"]
    assert xyz.shape == ref_xyz.shape
    assert np.array_equal(xyz.view(np.uint64), ref_xyz.view(np.uint64)), "XYZ not bit-exact"
    assert np.array_equal(rgb, store[f"{prefix}_rgb"])
    ref_dist = store[f"{prefix}_dist"]
    # keep-mask parity is the claim; dist bits document the BLAS order (OpenBLAS here)
    assert np.array_equal(dist < 0.05, ref_dist < 0.05)
    assert np.max(np.abs(dist - ref_dist), initial=0) <= 4e-15
    n, n1, n2 = r["counts"]
    assert n == len(ref_xyz)
    assert n1 == len(store[f"{prefix}_keep_idx"])
    assert n2 == len(store[f"{prefix}_keep2_idx"])
    assert np.array_equal(r["hist"], store[f"{prefix}_hist"])
    assert np.array_equal(r["pts"].reshape(-1, 1, 2), store[f"{prefix}_plane_points"])
    assert np.array_equal(r["xyz2"], ref_xyz[store[f"{prefix}_keep2_idx"]])
    return dist, ref_dist


@pytest.mark.parametrize("k", [0, 1, 2])
def test_sparse_frames_c_oracle(golden, k):
    disp, bgr = sparse_frame(golden, k)
    _check_chain(f"f{k}", golden.sparse, disp, bgr, np.array(golden.meta["plane_abc"]))


@pytest.mark.parametrize("k", [0, 1, 2])
def test_crops_c_oracle(golden, k):
    c = golden.crops
    dist, ref = _check_chain(f"c{k}", c, c[f"c{k}_disp"], c[f"c{k}_bgr"], c[f"c{k}_abc"])
    # the fma order restated in the oracle is bit-identical to the reference's np.dot here
    assert np.array_equal(dist, ref)


@pytest.mark.parametrize("fid", ["0", "1", "4095", "0r"])
def test_full_frames_step2_digests(golden, fid):
    m = golden.meta["full_frames_step2"][fid]
    disp, bgr = oracle.synth_frame(0 if fid == "0r" else int(fid))
    assert oracle.digest(disp) == m["disp"] and oracle.digest(bgr) == m["bgr"]
    xyz, rgb = oracle.project(disp, bgr, 2)
    assert oracle.digest(xyz) == m["xyz"] and oracle.digest(rgb) == m["rgb"]
    assert oracle.digest(oracle.project(disp, None, 2)[0]) == m["mask_xyz"]
    r = oracle.pipeline_frame(disp, bgr, 2, abc=np.array(m["abc"]))
    assert r["counts"] == (m["n"], m["n_kept"], m["n_kept2"])
    assert oracle.digest(r["hist"]) == m["hist"]
    assert oracle.digest(r["pts"].reshape(-1, 1, 2)) == m["plane_points"]


def test_generator_twins_agree():
    for fid in (0, 3, 4095, 32767):
        d1, b1 = oracle.synth_frame(fid)
        d2, b2 = osynth.frame(fid)
        assert np.array_equal(d1, d2) and np.array_equal(b1, b2)


def test_hue_lut_matches_reference_digest(golden):
    lut = oracle.hue_lut()
    assert oracle.digest(lut) == golden.meta["hue_lut"]["digest"]
    rgb = golden.hue["rgb"]
    idx = (rgb[:, 0] << 16) | (rgb[:, 1] << 8) | rgb[:, 2]
    assert np.array_equal(lut[idx], golden.hue["bins"])
    for r, g, b, k in golden.meta["hue_kat"]:
        assert oracle.hue_bin(r, g, b) == k


def test_hue_python_int_trap_documented(golden):
    """Python-int channels change some keys (SURVEY §0 trap 3): the drop-in must hand numpy scalars."""
    assert not np.array_equal(golden.hue["bins"], golden.hue["bins_pyint"])


def test_delta_tables_match_reference_roundtrip(golden):
    dx, dy = oracle.delta_tables()
    ref_dx, ref_dy = golden.deltas["dx_even"], golden.deltas["dy_even"]
    assert np.array_equal(dx.T[0:1023:2, 1:], ref_dx[0:1023:2, 1:])
    assert np.array_equal(dy.T[0:543:2, 1:], ref_dy[0:543:2, 1:])
    assert set(np.unique(dx)) <= {-1, 0} and set(np.unique(dy)) <= {-1, 0}


def test_cpu_loop_port_matches_reference_crops(golden):
    c = golden.crops
    for k in range(3):
        rows, kept, kept2, pp, hist = cpu_loop.chain(c[f"c{k}_disp"], c[f"c{k}_bgr"], c[f"c{k}_abc"])
        xyz = np.array([r[:3] for r in rows], np.float64)
        assert np.array_equal(xyz.view(np.uint64), c[f"c{k}_xyz"].view(np.uint64))
        assert len(kept) == len(c[f"c{k}_keep_idx"])
        assert np.array_equal(pp, c[f"c{k}_plane_points"])
        h = np.zeros(1024, np.uint32)
        for key, v in hist.items():
            h[cpu_loop.key_to_bin(key)] = v
        assert np.array_equal(h, c[f"c{k}_hist"])


def test_cpu_loop_port_matches_reference_sparse(golden):
    abc = np.array(golden.meta["plane_abc"])
    for k in range(3):
        disp, bgr = sparse_frame(golden, k)
        rows, kept, kept2, pp, hist = cpu_loop.chain(disp, bgr, abc)
        assert np.array_equal(pp, golden.sparse[f"f{k}_plane_points"])
        assert type(rows[0][3]) is np.uint8 and type(rows[0][0]) is np.float64


def test_cpu_loop_frame0_digest(golden):
    """The CPU port on synthetic frame 0 (the bench's config-1 input) gives the reference's XYZ digest,
    counts and planePoints digest (tests/golden/digests.json)."""
    import hashlib

    import oracle
    disp, bgr = oracle.synth_frame(0)
    rows, kept, kept2, pp, _ = cpu_loop.chain(disp, bgr, oracle.synthetic_plane())
    xyz = np.array([r[:3] for r in rows], np.float64)
    assert hashlib.sha256(xyz.tobytes()).hexdigest()[:16] == "4e8146c117e8d5f0"
    assert (len(rows), len(kept), len(kept2)) == (74200, 69341, 63826)
    assert hashlib.sha256(np.ascontiguousarray(pp).tobytes()).hexdigest()[:16] == "b6f5c4e7d5962a47"
