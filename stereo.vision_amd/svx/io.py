"""PNG ingest of the stereo pairs and masks: cv2.imread for the reference's files.

The reference reads its masks at import (functions.py:29-35, cv2.IMREAD_GRAYSCALE) and each stereo pair in
loadImages (functions.py:52-55, cv2.imread's default IMREAD_COLOR); getImagePaths (:41-50) pairs "_L" with "_R"
file names. OpenCV is absent here, so this reads 8-bit, non-interlaced PNGs itself: the chunks and zlib inflate in
Python, the scanline filters in libsvx (sv_png_unfilter, C ABI, host code), then OpenCV's PNG decoder's channel
handling:

* IMREAD_COLOR -> H x W x 3 BGR (alpha stripped, not composited; grey replicated; palette expanded);
* IMREAD_GRAYSCALE -> H x W (alpha stripped; a colour image through libpng's rgb_to_gray with OpenCV's
  coefficients 0.299 / 0.587, i.e. (9797 R + 19234 G + 3737 B) >> 15 where R, G, B differ, else R);
* IMREAD_UNCHANGED -> 1, 3 or 4 channels as OpenCV's decoder chooses them: grey 1; RGB and palette 3, or 4 with
  a tRNS chunk (alpha from it); grey + alpha 4 (BGRA, the grey replicated); RGBA 4; colour in BGR(A) order;
  uint16 for 16-bit files.

Parity: exact for the lossless decode (tests/test_io_cpu.py round-trips every filter type, colour type, bit
depth and Adam7 interlacing); the grey conversion restates libpng's published arithmetic and is unpinned against
OpenCV itself (absent; the reference's masks are black and white, where every formula gives the same bytes). A
corrupt file gives None, as cv2.imread does; a 16-bit colour file read as IMREAD_GRAYSCALE raises
NotImplementedError.
"""
import os
import struct
import zlib

import numpy as np

from . import _abi

IMREAD_UNCHANGED = -1
IMREAD_GRAYSCALE = 0
IMREAD_COLOR = 1

_SIG = b"\x89PNG\r\n\x1a\n"
_CHANNELS = {0: 1, 2: 3, 3: 1, 4: 2, 6: 4}   # PNG colour type -> samples a pixel
_DEPTHS = {0: (1, 2, 4, 8, 16), 2: (8, 16), 3: (1, 2, 4, 8), 4: (8, 16), 6: (8, 16)}
_CRITICAL = (b"IHDR", b"PLTE", b"IDAT", b"IEND")
# Adam7 passes: (x0, y0, dx, dy)
_ADAM7 = ((0, 0, 8, 8), (4, 0, 8, 8), (0, 4, 4, 8), (2, 0, 4, 4), (0, 2, 2, 4), (1, 0, 2, 2), (0, 1, 1, 2))


class PngCorrupt(ValueError):
    """The file is not a decodable PNG (cv2.imread returns None for it)."""


def _samples(raw, h, w, ch, depth):
    """unfiltered scanlines (h x rowbytes) -> (h, w, ch) samples: uint8 for depth <= 8, uint16 for 16."""
    if depth == 8:
        return raw.reshape(h, w, ch)
    if depth == 16:
        return raw.reshape(h, w * ch, 2).view(">u2").reshape(h, w, ch).astype(np.uint16)
    per = 8 // depth   # samples a byte, the first in the high bits
    bits = np.unpackbits(raw, axis=1).reshape(h, -1, depth)
    vals = (bits * (1 << np.arange(depth - 1, -1, -1, dtype=np.uint8))).sum(axis=2, dtype=np.uint16)
    assert vals.shape[1] == raw.shape[1] * per
    return vals[:, : w * ch].astype(np.uint8).reshape(h, w, ch)


def _unfilter(data, h, rowbytes, bpp):
    if len(data) < h * (rowbytes + 1):
        raise PngCorrupt("truncated image data")
    src = np.ascontiguousarray(np.frombuffer(data, np.uint8, count=h * (rowbytes + 1)))
    out = np.empty((h, rowbytes), np.uint8)
    if h:
        rc = _abi.lib().sv_png_unfilter(_abi.ptr(src), h, rowbytes, bpp, _abi.ptr(out))
        if rc != 0:
            raise PngCorrupt("bad scanline filter type")
    return out


def _read_png(path):
    """(samples H x W x C as stored — uint8, or uint16 at depth 16 — with sub-byte grey scaled to 8 bits and
    palette indices expanded to RGB(A), colour type of the result, tRNS key or None, depth). Raises PngCorrupt."""
    with open(path, "rb") as fh:
        data = fh.read()
    if data[:8] != _SIG:
        raise PngCorrupt(f"{path}: not a PNG file")
    pos, ihdr, idat, plte, trns = 8, None, [], None, None
    while True:
        if pos + 12 > len(data):
            raise PngCorrupt(f"{path}: truncated chunk")
        ln, typ = struct.unpack(">I4s", data[pos:pos + 8])
        body = data[pos + 8:pos + 8 + ln]
        if len(body) < ln or pos + 12 + ln > len(data):
            raise PngCorrupt(f"{path}: truncated chunk")
        crc = struct.unpack(">I", data[pos + 8 + ln:pos + 12 + ln])[0]
        good = zlib.crc32(typ + body) & 0xFFFFFFFF == crc
        if not good and typ in _CRITICAL:   # libpng: an error for critical chunks, ancillary ones are dropped
            raise PngCorrupt(f"{path}: CRC error in {typ.decode('latin-1')}")
        if typ == b"IHDR":
            ihdr = struct.unpack(">IIBBBBB", body)
        elif typ == b"PLTE":
            plte = np.frombuffer(body, np.uint8)[: len(body) // 3 * 3].reshape(-1, 3)
        elif typ == b"tRNS" and good:
            trns = np.frombuffer(body, np.uint8)
        elif typ == b"IDAT":
            idat.append(body)
        elif typ == b"IEND":
            break
        pos += 12 + ln
    if ihdr is None:
        raise PngCorrupt(f"{path}: no IHDR chunk")
    W, H, depth, ctype, _comp, _filt, interlace = ihdr
    if ctype not in _CHANNELS or depth not in _DEPTHS[ctype] or interlace > 1 or W == 0 or H == 0:
        raise PngCorrupt(f"{path}: bad IHDR (colour type {ctype}, depth {depth}, interlace {interlace})")
    ch = _CHANNELS[ctype]
    try:
        raw = zlib.decompress(b"".join(idat))
    except zlib.error as e:
        raise PngCorrupt(f"{path}: {e}") from None
    bpp = max(1, ch * depth // 8)   # the filters' left neighbour, in bytes
    px = np.zeros((H, W, ch), np.uint16 if depth == 16 else np.uint8)
    passes = _ADAM7 if interlace else ((0, 0, 1, 1),)
    off = 0
    for x0, y0, dx, dy in passes:
        pw, ph = (W - x0 + dx - 1) // dx, (H - y0 + dy - 1) // dy
        if pw <= 0 or ph <= 0:
            continue   # an empty pass has no scanlines (and no filter bytes)
        rowbytes = (pw * ch * depth + 7) // 8
        rows = _unfilter(raw[off:], ph, rowbytes, bpp)
        off += ph * (rowbytes + 1)
        px[y0::dy, x0::dx] = _samples(rows, ph, pw, ch, depth)
    if ctype == 0 and depth < 8:   # png_set_expand_gray_1_2_4_to_8: 0..2^b - 1 scaled to 0..255
        px = (px.astype(np.uint16) * (255 // ((1 << depth) - 1))).astype(np.uint8)
    key = None
    if ctype == 3:   # palette: indices -> RGB, or RGBA when the file gives palette alpha
        if plte is None or len(plte) == 0:
            raise PngCorrupt(f"{path}: palette image without PLTE")
        # libpng keeps a zero-filled 256-entry palette (alpha 255 past tRNS), so an index past PLTE decodes black
        pal = np.zeros((256, 3), np.uint8)
        pal[:min(len(plte), 256)] = plte[:256]
        idx = px[..., 0]
        rgb = pal[idx]
        if trns is not None and len(trns):
            alpha = np.full(256, 255, np.uint8)
            alpha[:min(len(trns), len(plte), 256)] = trns[:min(len(plte), 256)]
            return np.dstack([rgb, alpha[idx]]), 6, None, 8
        return rgb, 2, None, 8
    if trns is not None and ctype in (0, 2) and len(trns) >= 2 * ch:
        key = np.frombuffer(trns[: 2 * ch].tobytes(), ">u2").astype(np.uint16)   # the transparent sample value(s)
        if depth < 8:
            key = key * (255 // ((1 << depth) - 1))
    return px, ctype, key, depth


def _rgb_to_gray(rgb):
    """libpng's png_do_rgb_to_gray for 8 bits without gamma, with OpenCV's png_set_rgb_to_gray(1, 0.299, 0.587):
    coefficients 29900 * 32768 // 100000 = 9797, 58700 * 32768 // 100000 = 19234, blue 32768 - both = 3737;
    (rc R + gc G + bc B) >> 15, truncated, where the channels differ; the channel itself where they are equal."""
    r, g, b = (rgb[..., i].astype(np.uint32) for i in range(3))
    y = ((9797 * r + 19234 * g + 3737 * b) >> 15).astype(np.uint8)
    same = (r == g) & (r == b)
    return np.where(same, rgb[..., 0], y)


def imread(path, flags=IMREAD_COLOR):
    """cv2.imread(path, flags) for PNG files (functions.py:29-34, :55), with OpenCV's PNG decoder's rules
    (grfmt_png.cpp): a missing, unreadable or corrupt file (bad signature, CRC error in a critical chunk, truncated
    or undecodable data) returns None. Colour types, bit depths 1-16 and Adam7 interlacing are decoded; 16-bit
    samples are kept by IMREAD_UNCHANGED (uint16) and cut to their high byte otherwise (png_set_strip_16), except a
    16-bit colour file read as IMREAD_GRAYSCALE (libpng's 16-bit grey conversion is not restated:
    NotImplementedError)."""
    if not os.path.isfile(path):
        return None
    try:
        px, ctype, key, depth = _read_png(path)
    except (PngCorrupt, OSError):
        return None
    has_alpha = ctype in (4, 6)
    colour = ctype in (2, 6)
    if flags == IMREAD_UNCHANGED:
        # OpenCV's m_type: 4 channels for colour or grey with alpha and for RGB / palette with tRNS, else 3 or 1
        if ctype == 2 and key is not None:   # png_set_tRNS_to_alpha: 0 where the pixel equals the key
            a = np.where(np.all(px == key.astype(px.dtype), axis=2), 0, 255 if depth != 16 else 65535)
            px = np.dstack([px, a.astype(px.dtype)])
            has_alpha = True
        if colour:
            out = px[..., [2, 1, 0] + ([3] if has_alpha else [])]
        elif has_alpha:   # grey + alpha -> BGRA (png_set_gray_to_rgb)
            out = px[..., [0, 0, 0, 1]]
        else:
            out = px[..., 0]
        return np.ascontiguousarray(out)
    if depth == 16:
        if flags == IMREAD_GRAYSCALE and colour:
            raise NotImplementedError(f"{path}: 16-bit colour PNG as IMREAD_GRAYSCALE (libpng's 16-bit rgb_to_gray)")
        px = (px >> 8).astype(np.uint8)   # png_set_strip_16
    if flags == IMREAD_GRAYSCALE:
        if colour:
            return np.ascontiguousarray(_rgb_to_gray(px[..., :3]))
        return np.ascontiguousarray(px[..., 0])
    # IMREAD_COLOR (and any other flag cv2 treats as colour): BGR, alpha stripped, grey replicated
    if colour:
        return np.ascontiguousarray(px[..., [2, 1, 0]])
    return np.ascontiguousarray(np.repeat(px[..., :1], 3, axis=2))


def getImagePaths(filename_l, path_dir_l, path_dir_r):  # noqa: N802 (reference signature)
    """functions.py:41-50: the left file's right partner ("_L" -> "_R"), both joined to their directories, or
    False when the left name is not a PNG or the right file does not exist."""
    filename_right = filename_l.replace("_L", "_R")
    full_l = os.path.join(path_dir_l, filename_l)
    full_r = os.path.join(path_dir_r, filename_right)
    if (".png" in filename_l) and os.path.isfile(full_r):
        return (full_l, full_r)
    return False


def loadImages(image_paths):  # noqa: N802 (reference signature)
    """functions.py:52-55: both images of a pair as BGR (cv2.imread's default)."""
    filename_l, filename_r = image_paths
    return (imread(filename_l), imread(filename_r))


def load_masks(mask_dir):
    """functions.py:29-35: the reference's masks (IMREAD_GRAYSCALE) and carmask = cv2.bitwise_and(car_front_mask,
    car_front_mask, mask=view_range), i.e. car_front_mask where view_range != 0, else 0. A missing file gives None
    (plane_sample.png is absent from the reference's masks/, as functions.py:34 then loads None)."""
    names = ("disparity_cap", "road_threshold_mask", "car_front_mask", "black", "view_range", "plane_sample")
    m = {n: imread(os.path.join(mask_dir, n + ".png"), IMREAD_GRAYSCALE) for n in names}
    car, view = m["car_front_mask"], m["view_range"]
    m["carmask"] = None if car is None or view is None else np.where(view != 0, car, 0).astype(np.uint8)
    return m
