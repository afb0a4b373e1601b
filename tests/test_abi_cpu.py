"""CPU-only checks of the boundary: libsvx.so loads, exports every symbol that
include/svx.h declares, the ctypes table matches, and the host-side drop-in
logic behaves (no compute calls: there is no GPU here)."""
import os
import re
import subprocess

import numpy as np
import pytest

from conftest import REPO

HEADER = os.path.join(REPO, "include", "svx.h")


def declared_symbols():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(sv_[a-z0-9_]+)\s*\(", src)))


def test_library_exports_every_declared_symbol():
    from svx import _abi
    lib = _abi.LIB_PATH
    assert os.path.exists(lib), "run __graft_entry__.build() first"
    out = subprocess.run(["nm", "-D", "--defined-only", lib], capture_output=True, text=True,
                         check=True).stdout
    exported = {ln.split()[-1] for ln in out.splitlines() if " T " in ln}
    missing = [s for s in declared_symbols() if s not in exported]
    assert not missing, missing


def test_ctypes_table_covers_header():
    from svx import _abi
    assert set(declared_symbols()) == set(_abi.SIGNATURES)
    lib = _abi.lib()
    for name in _abi.SIGNATURES:
        assert getattr(lib, name) is not None
    assert _abi.lib().sv_version().decode().startswith("svx")


def test_library_is_gfx950():
    """The fat binary embeds gfx950 code objects (bundle id amdgcn-amd-amdhsa--gfx950)."""
    from svx import _abi
    blob = open(_abi.LIB_PATH, "rb").read()
    assert b"amdgcn-amd-amdhsa--gfx950" in blob


def test_release_library_reads_no_knobs():
    """The release libsvx.so carries no SVX_* knob (A/B selectors, placement probes,
    ablations that make results invalid): they are compiled only into the diagnostic
    libsvx_diag.so (-DSVX_DIAG, tools/prof.py). getenv itself may be linked (the HIP
    runtime's own), but no SVX_ name is in the binary for it to read."""
    from svx import _abi
    blob = open(_abi.LIB_PATH, "rb").read()
    assert b"SVX_" not in blob
    diag = os.path.join(os.path.dirname(_abi.LIB_PATH), "libsvx_diag.so")
    if os.path.exists(diag):
        dblob = open(diag, "rb").read()
        assert b"SVX_ABLATE" in dblob and b"SVX_RANSAC_ABLATE" in dblob


def test_diagnostic_library_loads_with_its_probes():
    """The diagnostic build loads (every symbol it uses resolves) and exports the evaluation's phase clocks
    (tools/_probe_eval_phases.py); the release build does not export them."""
    import ctypes
    from svx import _abi
    diag = os.path.join(os.path.dirname(_abi.LIB_PATH), "libsvx_diag.so")
    if not os.path.exists(diag):
        pytest.skip("diagnostic library not built")
    d = ctypes.CDLL(diag)
    assert hasattr(d, "sv_diag_eval_phases") and hasattr(d, "sv_batch_create")
    assert not hasattr(_abi.lib(), "sv_diag_eval_phases")


def test_no_device_errors_are_raised_not_faked():
    """Without a GPU every compute entry point must fail loudly (no CPU fallback)."""
    import svx
    from svx import SvxError, batch, dropin
    if svx.device_count() > 0:
        pytest.skip("GPU present")
    with pytest.raises(SvxError):
        dropin.projectDisparityTo3d(np.ones((8, 8), np.uint8), 128)
    with pytest.raises(SvxError):
        dropin.project3DPointsTo2DImagePoints([[1.0, 2.0, 3.0]])
    with pytest.raises(SvxError):
        batch.Batch(1)


def test_dropin_argument_checks_before_device():
    from svx import dropin
    with pytest.raises(TypeError):
        dropin.projectDisparityTo3d(np.zeros((4, 4), np.float64), 128)
    with pytest.raises(ValueError):
        dropin.projectDisparityTo3d(np.zeros((4, 4, 2), np.uint8), 128)
    assert len(dropin.project3DPointsTo2DImagePoints([])) == 0
    assert np.array(dropin.project3DPointsTo2DImagePoints([]), np.int32).reshape((-1, 1, 2)).shape == (0, 1, 2)


def test_install_patches_module_attributes():
    import types

    from svx import dropin
    m = types.SimpleNamespace(camera_focal_length_px=1.0, stereo_camera_baseline_m=2.0,
                              image_centre_w=3.0, image_centre_h=4.0,
                              projectDisparityTo3d=None, project3DPointsTo2DImagePoints=None)
    dropin.install(m)
    try:
        assert m.projectDisparityTo3d is dropin.projectDisparityTo3d
        assert m.project3DPointsTo2DImagePoints is dropin.project3DPointsTo2DImagePoints
        assert m.project_disparity_to_3d is dropin.projectDisparityTo3d
        assert m.project_3D_points_to_2D is dropin.project3DPointsTo2DImagePoints
        cam = dropin._camera()
        assert (cam.f, cam.B, cam.cw, cam.ch) == (1.0, 2.0, 3.0, 4.0)
    finally:
        dropin.uninstall()
    cam = dropin._camera()
    assert (cam.f, cam.B, cam.cw, cam.ch) == dropin.DEFAULT_CAMERA


def test_install_default_is_the_pinned_set():
    """install(functions) replaces only the functions pinned against the reference's own outputs; the
    restatements of OpenCV (disparity, greyscale, fillDisparity, maskDisparity, and the PNG ingest getImagePaths /
    loadImages: functions.py:41-55,88-96,104-128,140-147,169-171) stay the module's originals unless
    install(.., unpinned=True)."""
    import types

    from svx import dropin
    orig = {name: (lambda *a, _n=name: _n) for name in dropin.PATCHED}
    m = types.SimpleNamespace(camera_focal_length_px=1.0, stereo_camera_baseline_m=2.0,
                              image_centre_w=3.0, image_centre_h=4.0, **orig)
    assert set(dropin.UNPINNED) == {"disparity", "greyscale", "fillDisparity", "maskDisparity", "getImagePaths",
                                    "loadImages"}
    dropin.install(m)
    try:
        for name in dropin.UNPINNED:
            assert getattr(m, name) is orig[name], name
        for name in dropin.PINNED:
            assert getattr(m, name) is not orig[name], name
    finally:
        dropin.uninstall()
    assert all(getattr(m, n) is orig[n] for n in dropin.PATCHED)
    dropin.install(m, unpinned=True)
    try:
        for name in dropin.PATCHED:
            assert getattr(m, name) is not orig[name], name
        assert m.maskDisparity is dropin.maskDisparity and m.disparity is dropin.disparity
    finally:
        dropin.uninstall()
    assert all(getattr(m, n) is orig[n] for n in dropin.PATCHED)


def test_header_cites_reference():
    src = open(HEADER).read()
    for cite in ("functions.py:178-198", "functions.py:201-209", "stereovision.py:84"):
        assert cite in src


def test_point_list_tracks_its_array():
    """The lazy row sequence projectDisparityTo3d returns (svx/points.py): a Sequence random.sample takes
    (functions.py:252,286), rows made on first read and the same objects afterwards (also through selections,
    as the reference's list comprehensions share rows), writes through rows reach the array, and a mutation
    turns it into a plain list that forgot the array."""
    import collections.abc
    import random
    from svx.dropin import PointList, as_points_array
    a = np.arange(12, dtype=np.float64).reshape(4, 3)
    pl = PointList(a)
    assert isinstance(pl, collections.abc.Sequence) and len(pl) == 4 and as_points_array(pl) is a
    assert pl[1] is pl[1] and pl[-1] is pl[3] and type(pl[0][0]) is np.float64
    with pytest.raises(IndexError):
        pl[4]
    pl[1][0] = 99.0                       # a write through a row view is a write to the array
    assert a[1, 0] == 99.0 and as_points_array(pl) is a
    rows = list(pl)
    assert len(rows) == 4 and all(r is pl[i] for i, r in enumerate(rows))
    sub = PointList.subset(pl, [3, 1])
    assert len(sub) == 2 and sub[0] is pl[3] and sub[1] is pl[1] and np.array_equal(sub.array(), a[[3, 1]])
    sub2 = PointList.subset(sub, [1])
    assert sub2[0] is pl[1] and np.array_equal(sub2.array(), a[[1]])
    sl = pl[1:3]
    assert len(sl) == 2 and sl[0] is pl[1] and np.array_equal(as_points_array(sl), a[1:3])
    pl.append(np.zeros(3))
    assert pl.array() is None and as_points_array(pl).shape == (5, 3) and pl[1] is rows[1]
    pl2 = PointList(a)
    del pl2[0]
    assert pl2.array() is None and np.array_equal(as_points_array(pl2), a[1:])
    assert len(random.Random(0).sample(PointList(a), 2)) == 2
    pl3 = PointList(a)
    assert PointList(np.zeros((0, 3))) == [] and not PointList(np.zeros((0, 3))) and pl3 == list(pl3)
    big = PointList(np.zeros((74200, 6)))
    assert len(random.Random(1).sample(big, 600)) == 600 and sum(r is not None for r in big._cache) == 600


def test_hue_keys_match_reference_strings():
    """svx.stages.bin_key(k) is the reference's str(round(h, 3)) for bin k, and every key the
    reference produced in tests/golden/stages.json is one of them (CPU only)."""
    import json
    import os

    import numpy as np

    from conftest import GOLDEN
    from svx import stages
    keys = [stages.bin_key(k) for k in range(1000)]
    assert keys == [str(round(np.float64(k / 1000), 3)) for k in range(1000)]
    fx = json.load(open(os.path.join(GOLDEN, "stages.json")))
    seen = {key for c in fx["crops"].values() for key, _ in c["hist_items"] + c["default_hist_items"]}
    assert seen <= set(keys) and len(seen) > 900


def test_loop_params_layout_matches_header(tmp_path):
    """svx._abi.LoopParams (ctypes) has the size and field offsets of include/svx.h's sv_loop_params (checked by
    compiling the header with the host C compiler)."""
    import ctypes
    import shutil
    import subprocess

    from svx import _abi
    cc = shutil.which("gcc") or shutil.which("cc")
    if cc is None:
        pytest.skip("no host C compiler")
    fields = [f for f, _ in _abi.LoopParams._fields_]
    src = tmp_path / "lp.c"
    src.write_text('#include <stdio.h>\n#include <stddef.h>\n#include "svx.h"\nint main(void){printf("%zu'
                   + "".join(" %zu" for _ in fields) + '\\n", sizeof(sv_loop_params)'
                   + "".join(f", offsetof(sv_loop_params, {f})" for f in fields) + ");return 0;}\n")
    exe = tmp_path / "lp"
    subprocess.check_call([cc, "-I", os.path.dirname(HEADER), str(src), "-o", str(exe)])
    got = [int(v) for v in subprocess.check_output([str(exe)]).split()]
    want = [ctypes.sizeof(_abi.LoopParams)] + [getattr(_abi.LoopParams, f).offset for f in fields]
    assert got == want
