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


def _filter_row(ft, row, prev, bpp):
    """one scanline filtered with type ft (PNG 1.2 §6), vectorised: every predictor reads raw bytes only"""
    x = np.frombuffer(row, np.uint8).astype(np.int16)
    b = np.frombuffer(prev, np.uint8).astype(np.int16) if prev is not None else np.zeros_like(x)
    a = np.concatenate([np.zeros(bpp, np.int16), x[:-bpp]])[: len(x)]
    c = np.concatenate([np.zeros(bpp, np.int16), b[:-bpp]])[: len(x)]
    if ft == 0:
        pred = np.zeros_like(x)
    elif ft == 1:
        pred = a
    elif ft == 2:
        pred = b
    elif ft == 3:
        pred = (a + b) >> 1
    else:   # Paeth: the neighbour nearest a + b - c, ties a, b, c
        p = a + b - c
        pa, pb, pc = np.abs(p - a), np.abs(p - b), np.abs(p - c)
        pred = np.where((pa <= pb) & (pa <= pc), a, np.where(pb <= pc, b, c))
    return bytes([ft]) + ((x - pred) & 0xFF).astype(np.uint8).tobytes()


ADAM7 = ((0, 0, 8, 8), (4, 0, 8, 8), (0, 4, 4, 8), (2, 0, 4, 4), (0, 2, 2, 4), (1, 0, 2, 2), (0, 1, 1, 2))


def _row_bytes(row, depth):
    """one scanline's samples (1-D, uint8 or uint16) as the file stores them"""
    if depth == 16:
        return row.astype(">u2").tobytes()
    if depth == 8:
        return row.astype(np.uint8).tobytes()
    per = 8 // depth
    v = np.zeros(-(-len(row) // per) * per, np.uint8)
    v[: len(row)] = row
    v = v.reshape(-1, per)
    return bytes((v << (8 - depth * (np.arange(per) + 1))).sum(axis=1, dtype=np.uint16).astype(np.uint8).tolist())


def write_png(path, samples, ctype, palette=None, trns=None, filters=(0, 1, 2, 3, 4), depth=8, interlace=0,
              corrupt=None):
    """samples: H x W x C as the file stores them (C per colour type; uint16 values at depth 16); rows cycle
    through `filters`; interlace 1 = Adam7; corrupt: "crc" (IDAT CRC) or "trunc" (data cut short)."""
    H, W, C = samples.shape
    bpp = max(1, C * depth // 8)
    raw = b""
    passes = ADAM7 if interlace else ((0, 0, 1, 1),)
    for x0, y0, dx, dy in passes:
        sub = samples[y0::dy, x0::dx]
        prev = None
        for y in range(sub.shape[0]):
            if sub.shape[1] == 0:
                break
            row = _row_bytes(sub[y].reshape(-1), depth)
            raw += _filter_row(filters[y % len(filters)], row, prev, bpp)
            prev = row

    def chunk(t, body, bad=False):
        crc = zlib.crc32(t + body) & 0xFFFFFFFF
        return struct.pack(">I", len(body)) + t + body + struct.pack(">I", crc ^ (1 if bad else 0))

    data = b"\x89PNG\r\n\x1a\n" + chunk(b"IHDR", struct.pack(">IIBBBBB", W, H, depth, ctype, 0, 0, interlace))
    if palette is not None:
        data += chunk(b"PLTE", palette.astype(np.uint8).tobytes())
    if trns is not None:
        data += chunk(b"tRNS", np.asarray(trns).astype(">u2" if ctype in (0, 2) else np.uint8).tobytes())
    z = zlib.compress(raw, 6)
    if corrupt == "trunc":
        z = z[: len(z) // 2]
    data += chunk(b"IDAT", z[: len(z) // 2]) + chunk(b"IDAT", z[len(z) // 2:], bad=corrupt == "crc")
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
    else:   # OpenCV's decoder: grey + alpha comes back as 4 channels, BGRA
        exp = px[..., [0, 0, 0, 1]] if alpha else px[..., 0]
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


def test_palette_index_past_plte_is_black(tmp_path):
    """An index past the PLTE entries decodes as libpng's zero-filled 256-entry palette gives it: black (and opaque
    past tRNS), not the last entry (the decoder had clamped the index)."""
    pal = np.array([[10, 20, 30], [40, 50, 60], [70, 80, 90]], np.uint8)
    idx = np.array([[[0], [2], [3], [200]], [[1], [255], [0], [2]]], np.uint8)
    p = str(tmp_path / "pal_short.png")
    write_png(p, idx, 3, palette=pal)
    full = np.zeros((256, 3), np.uint8)
    full[:3] = pal
    np.testing.assert_array_equal(sio.imread(p), full[idx[..., 0]][..., ::-1])
    q = str(tmp_path / "pal_short_a.png")
    write_png(q, idx, 3, palette=pal, trns=np.array([7, 8], np.uint8))
    un = sio.imread(q, sio.IMREAD_UNCHANGED)
    alpha = np.full(256, 255, np.uint8)
    alpha[:2] = (7, 8)
    np.testing.assert_array_equal(un[..., :3], full[idx[..., 0]][..., ::-1])
    np.testing.assert_array_equal(un[..., 3], alpha[idx[..., 0]])


def test_missing_and_corrupt_files_are_none(tmp_path):
    """cv2.imread returns None (it does not raise) for a file it cannot decode"""
    assert sio.imread(str(tmp_path / "absent.png")) is None
    bad = tmp_path / "bad.png"
    bad.write_bytes(b"not a png")
    assert sio.imread(str(bad)) is None
    px = np.random.default_rng(9).integers(0, 256, (7, 9, 3), dtype=np.uint8)
    for how in ("crc", "trunc"):
        p = str(tmp_path / f"{how}.png")
        write_png(p, px, 2, corrupt=how)
        assert sio.imread(p) is None, how
    ok = str(tmp_path / "ok.png")
    write_png(ok, px, 2)
    data = open(ok, "rb").read()
    open(ok, "wb").write(data[: len(data) - 20])   # cut inside the last chunks
    assert sio.imread(ok) is None


@pytest.mark.parametrize("depth", [1, 2, 4, 8, 16])
@pytest.mark.parametrize("interlace", [0, 1])
def test_grey_bit_depths_and_interlacing(tmp_path, depth, interlace):
    """png_set_expand_gray_1_2_4_to_8 (v * 255 / (2^b - 1)), 16-bit kept by IMREAD_UNCHANGED and cut to the high
    byte otherwise (png_set_strip_16), Adam7 interlacing on an odd size (empty passes included)"""
    rng = np.random.default_rng(depth + 10 * interlace)
    px = rng.integers(0, 1 << depth, (11, 13, 1)).astype(np.uint16 if depth == 16 else np.uint8)
    p = str(tmp_path / f"g{depth}.png")
    write_png(p, px, 0, depth=depth, interlace=interlace)
    un = sio.imread(p, sio.IMREAD_UNCHANGED)
    grey8 = (px[..., 0] >> 8).astype(np.uint8) if depth == 16 else (px[..., 0] * (255 // ((1 << depth) - 1))).astype(np.uint8)
    np.testing.assert_array_equal(un, px[..., 0] if depth == 16 else grey8)
    assert un.dtype == (np.uint16 if depth == 16 else np.uint8)
    np.testing.assert_array_equal(sio.imread(p, sio.IMREAD_GRAYSCALE), grey8)
    np.testing.assert_array_equal(sio.imread(p), np.repeat(grey8[..., None], 3, axis=2))


@pytest.mark.parametrize("depth", [1, 2, 4, 8])
def test_palette_bit_depths_interlaced(tmp_path, depth):
    rng = np.random.default_rng(depth)
    pal = rng.integers(0, 256, (1 << depth, 3), dtype=np.uint8)
    idx = rng.integers(0, 1 << depth, (9, 10, 1), dtype=np.uint8)
    p = str(tmp_path / f"p{depth}.png")
    write_png(p, idx, 3, palette=pal, depth=depth, interlace=1)
    np.testing.assert_array_equal(sio.imread(p), pal[idx[..., 0]][..., ::-1])


def test_rgb16_and_rgb_trns(tmp_path):
    rng = np.random.default_rng(4)
    px = rng.integers(0, 65536, (6, 7, 3)).astype(np.uint16)
    p = str(tmp_path / "rgb16.png")
    write_png(p, px, 2, depth=16, interlace=1)
    np.testing.assert_array_equal(sio.imread(p, sio.IMREAD_UNCHANGED), px[..., ::-1])
    np.testing.assert_array_equal(sio.imread(p), (px[..., ::-1] >> 8).astype(np.uint8))
    with pytest.raises(NotImplementedError):   # libpng's 16-bit grey conversion is not restated
        sio.imread(p, sio.IMREAD_GRAYSCALE)
    # an RGB tRNS key: IMREAD_UNCHANGED gives BGRA with alpha 0 exactly where the pixel is the key
    q8 = rng.integers(0, 4, (6, 7, 3), dtype=np.uint8) * 60
    key = q8[2, 3].astype(np.uint16)
    q = str(tmp_path / "rgb_trns.png")
    write_png(q, q8, 2, trns=key)
    un = sio.imread(q, sio.IMREAD_UNCHANGED)
    assert un.shape == (6, 7, 4)
    np.testing.assert_array_equal(un[..., :3], q8[..., ::-1])
    np.testing.assert_array_equal(un[..., 3], np.where(np.all(q8 == key, axis=2), 0, 255))
    np.testing.assert_array_equal(sio.imread(q), q8[..., ::-1])   # IMREAD_COLOR strips it


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


def test_against_pil_encoder_and_decoder(tmp_path):
    """An independent codec where one is importable (PIL, this container): files PIL writes (its own adaptive
    filters; modes 1, L, LA, P, RGB, RGBA) decode to PIL's pixels, and PIL decodes this file's Adam7-interlaced
    writer's files to the same pixels as svx.io."""
    Image = pytest.importorskip("PIL.Image")
    rng = np.random.default_rng(21)
    H, W = 37, 53
    smooth = (np.add.outer(np.arange(H), np.arange(W)) * 3 % 256).astype(np.uint8)   # filters other than None pay
    imgs = {
        "1": Image.fromarray(rng.integers(0, 2, (H, W)).astype(bool)),
        "L": Image.fromarray(smooth),
        "LA": Image.fromarray(np.dstack([smooth, rng.integers(0, 256, (H, W), dtype=np.uint8)]), "LA"),
        "RGB": Image.fromarray(np.dstack([smooth, smooth[::-1], rng.integers(0, 256, (H, W), dtype=np.uint8)])),
        "RGBA": Image.fromarray(rng.integers(0, 256, (H, W, 4), dtype=np.uint8)),
    }
    imgs["P"] = imgs["RGB"].quantize(colors=37)
    for mode, im in imgs.items():
        p = str(tmp_path / f"pil_{mode}.png")
        im.save(p)
        rgb = np.asarray(Image.open(p).convert("RGB"))
        np.testing.assert_array_equal(sio.imread(p), rgb[..., ::-1], err_msg=mode)
        if mode in ("1", "L"):
            np.testing.assert_array_equal(sio.imread(p, sio.IMREAD_GRAYSCALE), np.asarray(Image.open(p).convert("L")))
    for ctype, C in ((0, 1), (2, 3), (4, 2), (6, 4)):
        px = rng.integers(0, 256, (H, W, C), dtype=np.uint8)
        p = str(tmp_path / f"adam7_{ctype}.png")
        write_png(p, px, ctype, interlace=1)
        ref = np.asarray(Image.open(p).convert("RGB"))
        np.testing.assert_array_equal(sio.imread(p), ref[..., ::-1], err_msg=str(ctype))
