#!/usr/bin/env python3
"""Generate the golden fixtures by running the REFERENCE's own Python functions.

CONTAINER ONLY: needs /root/reference (absent on the GPU box). Run as

    PYTHONDONTWRITEBYTECODE=1 python3 -B tests/golden/make_golden.py

The reference imports cv2 at module level (functions.py:2, :26-35) but none of
the hot-path functions use it, so a stub module stands in for cv2. The
reference's functions then run UNMODIFIED; only their inputs/outputs are
saved here (data, never source):

* sparse.npz     — 3 sparse 544x1024 frames (edge values d in {1,2,254,255},
                   x in {0,474,475,1022,1023}, y in {0,1,262,542,543}, grey and
                   exact-hue-tie colours) through the whole chain of
                   stereovision.py:84,97-113.
* crops.npz      — the same chain on 96x512 crops of synthetic frames.
* digests.json   — digests/counts of the chain on full synthetic frames 0, 1,
                   4095 (step 2), the hue-bin LUT over all 2^24 colours, the
                   back-projection delta tables and known-answer hue values.
* hue_sample.npz — 8192 colours (random + exact-tie + grey) and their bins.
* deltas.npz     — dx[x][d] for even x and dy[y][d] for even y, measured
                   through the reference's own projection + back-projection.
"""
import hashlib
import json
import multiprocessing as mp
import os
import sys
import types

import numpy as np

REF = "/root/reference"
OUT = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(OUT))


def load_reference():
    if not os.path.isdir(REF):
        raise SystemExit("make_golden.py needs the reference at /root/reference (container only)")
    sys.dont_write_bytecode = True
    stub = types.ModuleType("cv2")
    stub.__getattr__ = lambda name: (lambda *a, **k: None)
    sys.modules["cv2"] = stub
    if REF not in sys.path:
        sys.path.insert(0, REF)
    import functions  # noqa: E402  (the reference, unmodified)
    return functions


def digest(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()[:16]


def key_to_bin(key):
    """str(round(h,3)) -> integer bin rint(h*1000) (one-to-one)."""
    return int(round(float(key) * 1000))


def run_chain(F, disp, bgr, abc, point_thr=0.05, hist_thr=10):
    """stereovision.py:84,97-113 with the reference functions, step 2."""
    points = F.projectDisparityTo3d(disp, 128, bgr)
    n = len(points)
    xyz = np.array([p[:3] for p in points], np.float64).reshape(-1, 3)
    rgb = np.array([p[3:6] for p in points], np.uint8).reshape(-1, 3)
    abc_col = np.asarray(abc, np.float64).reshape(3, 1)
    dist = F.calculatePointErrors(abc_col, points).reshape(-1) if n else np.zeros(0)
    kept = F.computePlanarThreshold(points, dist.reshape(-1, 1), point_thr)
    keep_idx = np.array([i for i in range(n) if dist[i] < point_thr], np.int64)
    assert len(keep_idx) == len(kept)
    hist = F.calculateColourHistogram(kept)
    hist_u32 = np.zeros(1024, np.uint32)
    for k, v in hist.items():
        hist_u32[key_to_bin(k)] = v
    kept2 = F.filterPointsByHistogram(kept, hist, hist_thr)
    kept_ids = {id(p): i for i, p in zip(keep_idx, kept)}
    keep2_idx = np.array([kept_ids[id(p)] for p in kept2], np.int64)
    pp = F.project3DPointsTo2DImagePoints(kept2)
    pp = np.array(pp, np.int32).reshape((-1, 1, 2))
    maskpoints = F.projectDisparityTo3d(disp, 128)
    mxyz = np.array([p[:3] for p in maskpoints], np.float64).reshape(-1, 3)
    return dict(xyz=xyz, rgb=rgb, dist=dist, keep_idx=keep_idx, hist=hist_u32,
                keep2_idx=keep2_idx, plane_points=pp, mask_xyz=mxyz)


def synth(fid, H=544, W=1024):
    sys.path.insert(0, REPO)
    from oracle import synth as S
    return S.frame(fid, H, W)


def synthetic_plane(F, horizon=200):
    """SURVEY §8d plane; `horizon` = the row where the synthetic disparity is 0."""
    f, B, ch = F.camera_focal_length_px, F.stereo_camera_baseline_m, F.image_centre_h
    k = 0.6
    return np.array([0.0, k / B, -k * (horizon - ch) / (f * B)], np.float64)


# a RANSAC-like plane (what RANSAC recovers on a similar frame)
RANSAC_LIKE = np.array([-0.007, 2.79, 0.457], np.float64)


def tie_colours(limit=2048):
    """Colours whose exact hue*1000 sits on a .5 boundary (rational tie)."""
    out = []
    rng = np.random.default_rng(7)
    while len(out) < limit:
        r, g, b = (int(v) for v in rng.integers(0, 256, 3))
        mx, mn = max(r, g, b), min(r, g, b)
        if mx == mn:
            continue
        rg = mx - mn
        if r == mx:
            n = g - b
        elif g == mx:
            n = 2 * rg + b - r
        else:
            n = 4 * rg + r - g
        n %= 6 * rg
        if (2000 * n) % (6 * rg * 2) == 6 * rg:  # 1000 n/(6 rg) = k + 1/2
            out.append((r, g, b))
    return out


def sparse_frames(F, abc):
    rng = np.random.default_rng(2024)
    H, W = 544, 1024
    palette = [(90, 100, 110), (91, 101, 112), (92, 100, 111), (93, 103, 110),
               (128, 128, 128), (0, 0, 0), (255, 255, 255), (255, 0, 0), (0, 255, 0),
               (0, 0, 255), (255, 128, 0)] + tie_colours(6)
    frames = []
    for k in range(3):
        disp0, bgr = synth(100 + k)
        disp = np.zeros((H, W), np.uint8)
        # plane-consistent pixels, mostly on the even grid, palette colours
        ys = rng.integers(200, H, 700)
        xs = rng.integers(0, W, 700)
        disp[ys, xs] = disp0[ys, xs]
        for y, x in zip(ys, xs):
            bgr[y, x] = palette[int(rng.integers(0, len(palette)))][::-1]
        # edge values
        for y in (0, 1, 262, 542, 543):
            for x in (0, 474, 475, 1022, 1023):
                disp[y, x] = (1, 2, 254, 255)[int(rng.integers(0, 4))]
        for i, d in enumerate((1, 2, 3, 127, 128, 253, 254, 255)):
            disp[300 + 2 * i, 100 + 2 * i] = d
        frames.append((disp, bgr))
    return frames


def hue_lut_chunk(args):
    r0, r1 = args
    F = load_reference()
    out = np.empty(((r1 - r0) << 16,), np.int16)
    u8 = np.uint8
    i = 0
    for r in range(r0, r1):
        for g in range(256):
            for b in range(256):
                out[i] = key_to_bin(F.BGRtoHSVHue((u8(r), u8(g), u8(b))))
                i += 1
    return out


def main():
    F = load_reference()
    abc = synthetic_plane(F)
    meta = {"reference": "thien/stereo.vision @ /root/reference", "python": sys.version.split()[0],
            "numpy": np.__version__, "plane_abc": abc.tolist(),
            "camera": [F.camera_focal_length_px, F.stereo_camera_baseline_m,
                       F.image_centre_w, F.image_centre_h]}

    # 1. sparse full-size frames
    arrays = {}
    for k, (disp, bgr) in enumerate(sparse_frames(F, abc)):
        r = run_chain(F, disp, bgr, abc)
        ys, xs = np.nonzero(disp)
        arrays[f"f{k}_pix"] = np.stack([ys, xs, disp[ys, xs]], 1).astype(np.int32)
        arrays[f"f{k}_pix_bgr"] = bgr[ys, xs]
        arrays[f"f{k}_frame_id"] = np.int64(100 + k)
        for name, v in r.items():
            arrays[f"f{k}_{name}"] = v
        print("sparse", k, len(r["xyz"]), len(r["keep_idx"]), len(r["keep2_idx"]))
    np.savez_compressed(os.path.join(OUT, "sparse.npz"), **arrays)

    # 2. crops of synthetic frames
    arrays = {}
    for k, (fid, y0, x0, ransac) in enumerate([(0, 176, 0, False), (4095, 200, 512, False),
                                               (7, 330, 256, True)]):
        disp, bgr = synth(fid)
        disp = np.ascontiguousarray(disp[y0:y0 + 96, x0:x0 + 512])
        bgr = np.ascontiguousarray(bgr[y0:y0 + 96, x0:x0 + 512])
        cabc = synthetic_plane(F, 200 - y0)
        if ransac:  # tilted, slightly wrong plane: many points near the threshold
            cabc[0] = -0.007
            cabc[1] *= 0.85
        r = run_chain(F, disp, bgr, cabc)
        arrays[f"c{k}_disp"] = disp
        arrays[f"c{k}_bgr"] = bgr
        arrays[f"c{k}_abc"] = cabc
        for name, v in r.items():
            if name != "mask_xyz":
                arrays[f"c{k}_{name}"] = v
        print("crop", k, len(r["xyz"]), len(r["keep_idx"]), len(r["keep2_idx"]))
    np.savez_compressed(os.path.join(OUT, "crops.npz"), **arrays)

    # 3. full synthetic frames, step 2
    full = {}
    for fid, plane in ((0, abc), (1, abc), (4095, abc), ("0r", RANSAC_LIKE)):
        disp, bgr = synth(0 if fid == "0r" else fid)
        r = run_chain(F, disp, bgr, plane)
        full[str(fid)] = {"abc": plane.tolist(), "disp": digest(disp), "bgr": digest(bgr), "xyz": digest(r["xyz"]),
                          "rgb": digest(r["rgb"]), "mask_xyz": digest(r["mask_xyz"]),
                          "n": len(r["xyz"]), "n_kept": len(r["keep_idx"]),
                          "n_kept2": len(r["keep2_idx"]), "hist": digest(r["hist"]),
                          "plane_points": digest(r["plane_points"]),
                          "keep_idx": digest(r["keep_idx"]), "keep2_idx": digest(r["keep2_idx"])}
        print("full", fid, full[str(fid)])
    meta["full_frames_step2"] = full

    # 4. hue: KATs, sample, full LUT digest through the reference BGRtoHSVHue
    u8 = np.uint8
    kat = [(0, 0, 0), (255, 0, 0), (0, 255, 0), (0, 0, 255), (90, 100, 110), (255, 128, 0), (200, 10, 100)]
    meta["hue_kat"] = [[r, g, b, key_to_bin(F.BGRtoHSVHue((u8(r), u8(g), u8(b))))] for r, g, b in kat]
    rng = np.random.default_rng(11)
    cols = [tuple(int(v) for v in c) for c in rng.integers(0, 256, (6000, 3))]
    cols += tie_colours(2048) + [(v, v, v) for v in range(0, 256, 2)][:144]
    cols = np.array(cols[:8192], np.int32)
    bins = np.array([key_to_bin(F.BGRtoHSVHue((u8(r), u8(g), u8(b)))) for r, g, b in cols], np.int16)
    # python-int inputs (the scalar-type trap of SURVEY §0): kept for the record
    bins_pyint = np.array([key_to_bin(F.BGRtoHSVHue((int(r), int(g), int(b)))) for r, g, b in cols], np.int16)
    np.savez_compressed(os.path.join(OUT, "hue_sample.npz"), rgb=cols, bins=bins, bins_pyint=bins_pyint)
    with mp.Pool(8) as pool:
        parts = pool.map(hue_lut_chunk, [(i, i + 8) for i in range(0, 256, 8)])
    lut = np.concatenate(parts)
    meta["hue_lut"] = {"digest": digest(lut), "layout": "int16, index R<<16|G<<8|B",
                       "max_bin": int(lut.max()), "n_bins": int(len(np.unique(lut)))}
    print("hue lut", meta["hue_lut"])

    # 5. back-projection deltas measured through the reference (even coords)
    H, W = 544, 1024
    img = np.zeros((510, W), np.uint8)
    for i in range(255):
        img[2 * i, :] = i + 1
    pts = F.projectDisparityTo3d(img, 128)
    back = np.array(F.project3DPointsTo2DImagePoints(pts), np.int32)
    dx = np.zeros((W, 256), np.int8)
    xs = np.tile(np.arange(0, W - 1, 2), 255)
    ds = np.repeat(np.arange(1, 256), len(range(0, W - 1, 2)))
    dx[xs, ds] = back[:, 0] - xs
    img = np.zeros((H, 512), np.uint8)
    for j in range(256):
        img[:, 2 * j] = min(j + 1, 255)
    pts = F.projectDisparityTo3d(img, 128)
    back = np.array(F.project3DPointsTo2DImagePoints(pts), np.int32)
    dy = np.zeros((H, 256), np.int8)
    ys = np.repeat(np.arange(0, H - 1, 2), 256)
    ds = np.tile(np.minimum(np.arange(1, 257), 255), len(range(0, H - 1, 2)))
    dy[ys, ds] = back[:, 1] - ys
    np.savez_compressed(os.path.join(OUT, "deltas.npz"), dx_even=dx, dy_even=dy)
    meta["deltas_even"] = {"dx": digest(dx), "dy": digest(dy), "dx_neg": int((dx == -1).sum()),
                           "dy_neg": int((dy == -1).sum())}
    print("deltas", meta["deltas_even"])

    with open(os.path.join(OUT, "digests.json"), "w") as fh:
        json.dump(meta, fh, indent=1, sort_keys=True)


if __name__ == "__main__":
    main()
