"""PNG ingest of the stereo pairs and masks: cv2.imread for the reference's files.

The reference reads its masks at import (functions.py:29-35, cv2.IMREAD_GRAYSCALE) and each stereo pair in
loadImages (functions.py:52-55, cv2.imread's default IMREAD_COLOR); getImagePaths (:41-50) pairs "_L" with "_R"
file names. OpenCV is absent here, so this reads 8-bit, non-interlaced PNGs itself: the chunks and zlib inflate in
Python, the scanline filters in libsvx (sv_png_unfilter, C ABI, host code), then OpenCV's PNG decoder's channel
handling:

* IMREAD_COLOR -> H x W x 3 BGR (alpha stripped, not composited; grey replicated; palette expanded);
* IMREAD_GRAYSCALE -> H x W (alpha stripped; a colour image through libpng's rgb_to_gray with OpenCV's
  coefficients 0.299 / 0.587, i.e. (9797 R + 19234 G + 3737 B) >> 15 where R, G, B differ, else R);
* IMREAD_UNCHANGED -> the file's channels, colour in BGR(A) order.

Parity: exact for the lossless decode (tests/test_io_cpu.py round-trips every filter type and colour type);
the grey conversion restates libpng's published arithmetic and is unpinned against OpenCV itself (absent; the
reference's masks are black and white, where every formula gives the same bytes). 16-bit and interlaced PNGs
raise ValueError.
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


def _read_png(path):
    """(H x W x C uint8 samples as stored: grey, grey+alpha, RGB, RGBA, or palette-expanded RGB(A))."""
    with open(path, "rb") as fh:
        data = fh.read()
    if data[:8] != _SIG:
        raise ValueError(f"{path}: not a PNG file")
    pos, ihdr, idat, plte, trns = 8, None, [], None, None
    while pos + 8 <= len(data):
        ln, typ = struct.unpack(">I4s", data[pos:pos + 8])
        body = data[pos + 8:pos + 8 + ln]
        if typ == b"IHDR":
            ihdr = struct.unpack(">IIBBBBB", body)
        elif typ == b"PLTE":
            plte = np.frombuffer(body, np.uint8).reshape(-1, 3)
        elif typ == b"tRNS":
            trns = np.frombuffer(body, np.uint8)
        elif typ == b"IDAT":
            idat.append(body)
        elif typ == b"IEND":
            break
        pos += 12 + ln
    if ihdr is None:
        raise ValueError(f"{path}: no IHDR chunk")
    W, H, depth, ctype, _comp, _filt, interlace = ihdr
    if ctype not in _CHANNELS:
        raise ValueError(f"{path}: unknown PNG colour type {ctype}")
    if depth != 8:
        raise ValueError(f"{path}: {depth}-bit PNG not supported (8-bit only)")
    if interlace:
        raise ValueError(f"{path}: interlaced PNG not supported")
    ch = _CHANNELS[ctype]
    raw = zlib.decompress(b"".join(idat))
    rowbytes = W * ch
    if len(raw) < H * (rowbytes + 1):
        raise ValueError(f"{path}: truncated image data")
    src = np.frombuffer(raw, np.uint8, count=H * (rowbytes + 1))
    out = np.empty((H, W, ch), np.uint8)
    _abi.call("sv_png_unfilter", _abi.ptr(np.ascontiguousarray(src)), H, rowbytes, ch, _abi.ptr(out))
    if ctype == 3:   # palette: indices -> RGB, or RGBA when the file gives palette alpha
        if plte is None:
            raise ValueError(f"{path}: palette image without PLTE")
        idx = out[..., 0]
        rgb = plte[np.minimum(idx, len(plte) - 1)]
        if trns is not None:
            alpha = np.full(len(plte), 255, np.uint8)
            alpha[:min(len(trns), len(plte))] = trns[:len(plte)]
            return np.dstack([rgb, alpha[np.minimum(idx, len(plte) - 1)]]), 6
        return rgb, 2
    return out, ctype


def _rgb_to_gray(rgb):
    """libpng's png_do_rgb_to_gray for 8 bits without gamma, with OpenCV's png_set_rgb_to_gray(1, 0.299, 0.587):
    coefficients 29900 * 32768 // 100000 = 9797, 58700 * 32768 // 100000 = 19234, blue 32768 - both = 3737;
    (rc R + gc G + bc B) >> 15, truncated, where the channels differ; the channel itself where they are equal."""
    r, g, b = (rgb[..., i].astype(np.uint32) for i in range(3))
    y = ((9797 * r + 19234 * g + 3737 * b) >> 15).astype(np.uint8)
    same = (r == g) & (r == b)
    return np.where(same, rgb[..., 0], y)


def imread(path, flags=IMREAD_COLOR):
    """cv2.imread(path, flags) for 8-bit PNG files (functions.py:29-34, :55). A missing or unreadable file
    returns None, as cv2.imread does."""
    if not os.path.isfile(path):
        return None
    px, ctype = _read_png(path)
    has_alpha = ctype in (4, 6)
    colour = ctype in (2, 6)
    if flags == IMREAD_UNCHANGED:
        if colour:
            bgr = px[..., [2, 1, 0] + ([3] if has_alpha else [])]
            return np.ascontiguousarray(bgr)
        return np.ascontiguousarray(px[..., 0] if not has_alpha else px)
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
