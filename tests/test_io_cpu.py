"""PNG ingest (svx.io: cv2.imread for the reference's pairs and masks, functions.py:29-35, 41-55), on the CPU.

A minimal encoder below writes PNGs with every scanline filter (None, Sub, Up, Average, Paeth) and every 8-bit
colour type; reading them back must give the samples exactly, with OpenCV's channel handling (BGR order, alpha
stripped, grey replicated, palette expanded) and libpng's rgb_to_gray for IMREAD_GRAYSCALE. The reference's own
masks are decoded when the reference checkout is present (this container only; never on the GPU box).
"""
import os
import struct
import zlib

import numpy as np
import pytest

from svx import io as sio

REF_MASKS = "/root/reference/masks"


def _paeth(a, b, c):
    p = a + b - c
    pa, pb, pc = abs(p - a), abs(p - b), abs(p - c)
    return a if pa <= pb and pa <= pc else (b if pb <= pc else c)


def _filter_row(ft, row, prev, bpp):
    out = bytearray(len(row))
    for i, x in enumerate(row):
        a = row[i - bpp] if i >= bpp else 0
        b = prev[i] if prev is not None else 0
        c = prev[i - bpp] if (prev is not None and i >= bpp) else 0
        pred = [0, a, b, (a + b) >> 1, _paeth(a, b, c)][ft]
        out[i] = (x - pred) & 0xFF
    return bytes([ft]) + bytes(out)


def write_png(path, samples, ctype, palette=None, trns=None, filters=(0, 1, 2, 3, 4)):
    """samples: H x W x C uint8 as the file stores them (C per colour type); rows cycle through `filters`."""
    H, W, C = samples.shape
    raw = b""
    prev = None
    for y in range(H):
        row = samples[y].reshape(-1).tobytes()
        raw += _filter_row(filters[y % len(filters)], row, prev, C)
        prev = row

    def chunk(t, body):
        return struct.pack(">I", len(body)) + t + body + struct.pack(">I", zlib.crc32(t + body) & 0xFFFFFFFF)

    data = b"\x89PNG\r\n\x1a\n" + chunk(b"IHDR", struct.pack(">IIBBBBB", W, H, 8, ctype, 0, 0, 0))
    if palette is not None:
        data += chunk(b"PLTE", palette.astype(np.uint8).tobytes())
    if trns is not None:
        data += chunk(b"tRNS", trns.astype(np.uint8).tobytes())
    z = zlib.compress(raw, 6)
    data += chunk(b"IDAT", z[: len(z) // 2]) + chunk(b"IDAT", z[len(z) // 2:])   # split over two IDATs
    data += chunk(b"IEND", b"")
    with open(path, "wb") as fh:
        fh.write(data)


@pytest.mark.parametrize("ctype,C", [(0, 1), (2, 3), (4, 2), (6, 4)])
def test_every_filter_and_colour_type_round_trips(tmp_path, ctype, C):
    rng = np.random.default_rng(ctype)
    px = rng.integers(0, 256, (13, 17, C), dtype=np.uint8)
    px[3] = px[2]                              # repeated rows (Up / Paeth with equal neighbours)
    px[5, :, :] = 255                          # saturated row (wrapping sums)
    p = str(tmp_path / f"t{ctype}.png")
    write_png(p, px, ctype)
    colour = ctype in (2, 6)
    alpha = ctype in (4, 6)
    un = sio.imread(p, sio.IMREAD_UNCHANGED)
    if colour:
        exp = px[..., [2, 1, 0] + ([3] if alpha else [])]
    else:
        exp = px if alpha else px[..., 0]
    np.testing.assert_array_equal(un, exp)
    bgr = sio.imread(p)
    np.testing.assert_array_equal(bgr, px[..., [2, 1, 0]] if colour else np.repeat(px[..., :1], 3, axis=2))
    grey = sio.imread(p, sio.IMREAD_GRAYSCALE)
    if colour:
        r, g, b = (px[..., i].astype(np.uint32) for i in range(3))
        y = ((9797 * r + 19234 * g + 3737 * b) >> 15).astype(np.uint8)
        np.testing.assert_array_equal(grey, np.where((r == g) & (r == b), px[..., 0], y))
    else:
        np.testing.assert_array_equal(grey, px[..., 0])


def test_palette_with_and_without_alpha(tmp_path):
    rng = np.random.default_rng(3)
    pal = rng.integers(0, 256, (20, 3), dtype=np.uint8)
    idx = rng.integers(0, 20, (9, 11, 1), dtype=np.uint8)
    p = str(tmp_path / "pal.png")
    write_png(p, idx, 3, palette=pal)
    np.testing.assert_array_equal(sio.imread(p), pal[idx[..., 0]][..., ::-1])
    trns = rng.integers(0, 256, 7, dtype=np.uint8)   # alpha for the first 7 entries, the rest opaque
    q = str(tmp_path / "pal_a.png")
    write_png(q, idx, 3, palette=pal, trns=trns)
    un = sio.imread(q, sio.IMREAD_UNCHANGED)
    alpha = np.full(20, 255, np.uint8)
    alpha[:7] = trns
    np.testing.assert_array_equal(un[..., :3], pal[idx[..., 0]][..., ::-1])
    np.testing.assert_array_equal(un[..., 3], alpha[idx[..., 0]])


def test_missing_file_is_none_and_bad_files_raise(tmp_path):
    assert sio.imread(str(tmp_path / "absent.png")) is None   # cv2.imread returns None
    bad = tmp_path / "bad.png"
    bad.write_bytes(b"not a png")
    with pytest.raises(ValueError):
        sio.imread(str(bad))


def test_image_pairing(tmp_path):
    """functions.py:41-50: "_L" -> "_R", a PNG on the left and an existing right file."""
    (tmp_path / "l").mkdir()
    (tmp_path / "r").mkdir()
    (tmp_path / "r" / "1506942473.484027_R.png").write_bytes(b"")
    got = sio.getImagePaths("1506942473.484027_L.png", str(tmp_path / "l"), str(tmp_path / "r"))
    assert got == (str(tmp_path / "l" / "1506942473.484027_L.png"), str(tmp_path / "r" / "1506942473.484027_R.png"))
    assert sio.getImagePaths("1506942473.484027_L.jpg", str(tmp_path / "l"), str(tmp_path / "r")) is False
    assert sio.getImagePaths("other_L.png", str(tmp_path / "l"), str(tmp_path / "r")) is False


def test_load_images_pairs_in_bgr(tmp_path):
    rng = np.random.default_rng(5)
    left = rng.integers(0, 256, (6, 8, 3), dtype=np.uint8)
    right = rng.integers(0, 256, (6, 8, 3), dtype=np.uint8)
    write_png(str(tmp_path / "a_L.png"), left, 2)
    write_png(str(tmp_path / "a_R.png"), right, 2)
    l, r = sio.loadImages(sio.getImagePaths("a_L.png", str(tmp_path), str(tmp_path)))
    np.testing.assert_array_equal(l, left[..., ::-1])
    np.testing.assert_array_equal(r, right[..., ::-1])


@pytest.mark.skipif(not os.path.isdir(REF_MASKS), reason="the reference checkout (this container only)")
def test_reference_masks_decode():
    """functions.py:29-35 on the reference's own masks: 1024 x 544 RGBA, black and white; plane_sample.png is
    absent (None, as the reference loads it); carmask covers 22.97 % of the pixels (measured)."""
    m = sio.load_masks(REF_MASKS)
    assert m["plane_sample"] is None
    for n in ("disparity_cap", "road_threshold_mask", "car_front_mask", "black", "view_range", "carmask"):
        assert m[n].shape == (544, 1024) and m[n].dtype == np.uint8, n
    cov = float(np.count_nonzero(m["carmask"])) / m["carmask"].size
    assert abs(cov - 0.2297) < 5e-4, cov
    # the carmask fixture the pre-pass and loop tests use (tests/golden/carmask.npz) is this mask, bit for bit
    from test_prepass_cpu import carmask
    np.testing.assert_array_equal(m["carmask"] != 0, carmask() != 0)
