"""Image<1>::read as the reference's Scene(const json&) uses it (image.h:84-95).

The source grid of `Scene(dict)` comes from the file named by "sourceValue"
(scene.h:31,36).  The reference dispatches on the extension, case-sensitively
(image.h:85-94, hasExtension :218-222): "pfm" -> readPFM, "png" -> readPNG,
anything else aborts (here: ValueError).

readPFM (image.h:105-149): rows are kept in FILE order -- buffer row i is file row
i, no bottom-to-top flip -- and every pixel goes through setFromRGB (:72-76): a
1-channel "Pf" value v is widened to rgb = (v, v, v) and the gray value is
0.299*r + 0.587*g + 0.114*b evaluated in DOUBLE, left to right, then stored as
float (so even a 1-channel value is not always returned unchanged).

readPNG (image.h:151-171): stb_image 2.28 (deps/stb/stb_image.h) decodes with
req_comp = 1: gray depths < 8 scaled by 0xff/0x55/0x11 (:4647,4783), palettes
expanded, 16-bit samples reduced to gray (stbi__compute_y_16, :1801) and then to 8
bits by >> 8 (:1198), colour to gray by (77 r + 150 g + 29 b) >> 8
(stbi__compute_y, :1744), alpha dropped (:1783-1786).  Each byte becomes
int(byte) / 255.0f in float (:166).  Rows top to bottom (no flip on load).
"""
import struct
import zlib

import numpy as np

__all__ = ["read_image", "read_pfm", "read_png"]


def _has_extension(filename, ext):
    # image.h:218-222: the text after the last '.', compared case-sensitively
    return filename[filename.rfind(".") + 1:] == ext


def read_image(path):
    """Image<1>(filename): float32 array [h, w], row i = the reader's row i."""
    path = str(path)
    if _has_extension(path, "pfm"):
        return read_pfm(path)
    if _has_extension(path, "png"):
        return read_png(path)
    raise ValueError(f"{path} not supported. Use PNG or PFM file format.")


def _gray_double(r, g, b):
    # setFromRGB, DIM == 1 (image.h:75): double products, left-to-right sum, float store
    r, g, b = (np.asarray(c, np.float32).astype(np.float64) for c in (r, g, b))
    return ((0.299 * r + 0.587 * g) + 0.114 * b).astype(np.float32)


class _Stream:
    """The operator>> tokenisation readPFM uses (whitespace-skipping chars/ints/floats)."""

    def __init__(self, data):
        self.d, self.i = data, 0

    def _skip_ws(self):
        while self.i < len(self.d) and self.d[self.i:self.i + 1].isspace():
            self.i += 1

    def char(self):
        self._skip_ws()
        if self.i >= len(self.d):
            return ""
        c = chr(self.d[self.i])
        self.i += 1
        return c

    def token(self, allowed):
        self._skip_ws()
        j = self.i
        while j < len(self.d) and chr(self.d[j]) in allowed:
            j += 1
        tok, self.i = self.d[self.i:j].decode(), j
        return tok


def read_pfm(path):
    with open(path, "rb") as f:
        data = f.read()
    s = _Stream(data)
    if s.char() != "P":
        raise ValueError(f"Invalid PFM file detected while reading {path}")
    channels = 3 if s.char() == "F" else 1  # image.h:120-121
    try:
        w = int(s.token("+-0123456789"))
        h = int(s.token("+-0123456789"))
        scale = float(s.token("+-0123456789.eEinfINFnaN"))
    except ValueError:
        raise ValueError(f"{path}: malformed PFM header") from None
    if w <= 0 or h <= 0:
        raise ValueError(f"{path}: bad PFM size {w}x{h}")
    s.i += 1  # file.ignore(1)
    little = scale < 0  # machine is little-endian: flip byte order iff the file is big-endian
    n = w * h * channels
    raw = data[s.i:s.i + 4 * n]
    vals = np.zeros(n, np.float32)  # a short file leaves the tail of tmpBuffer zero (image.h:132-133)
    m = len(raw) // 4
    vals[:m] = np.frombuffer(raw[:4 * m], "<f4" if little else ">f4")
    if channels == 3:
        px = vals.reshape(h, w, 3)
        return _gray_double(px[..., 0], px[..., 1], px[..., 2])
    px = vals.reshape(h, w)
    return _gray_double(px, px, px)


# ---------------------------------------------------------------- PNG (stb_image 2.28)

_ADAM7 = ((0, 0, 8, 8), (4, 0, 8, 8), (0, 4, 4, 8), (2, 0, 4, 4), (0, 2, 2, 4), (1, 0, 2, 2), (0, 1, 1, 2))
_CHANNELS = {0: 1, 2: 3, 3: 1, 4: 2, 6: 4}


def _unfilter(buf, width, height, bpp, stride):
    """Undo the per-scanline PNG filters (None/Sub/Up/Average/Paeth)."""
    out = np.zeros((height, stride), np.uint8)
    prev = np.zeros(stride, np.int32)
    pos = 0
    for y in range(height):
        ftype = buf[pos]
        line = np.frombuffer(buf, np.uint8, stride, pos + 1).astype(np.int32)
        pos += 1 + stride
        if ftype == 0:
            cur = line
        elif ftype == 2:
            cur = (line + prev) & 255
        elif ftype == 1:  # Sub: a running sum per byte lane
            cur = line.copy()
            for k in range(bpp):
                cur[k::bpp] = np.cumsum(line[k::bpp]) & 255
        else:
            cur = line.copy()
            for i in range(stride):
                a = cur[i - bpp] if i >= bpp else 0
                if ftype == 3:
                    cur[i] = (cur[i] + ((a + prev[i]) >> 1)) & 255
                elif ftype == 4:
                    b, c = prev[i], (prev[i - bpp] if i >= bpp else 0)
                    p = a + b - c
                    pa, pb, pc = abs(p - a), abs(p - b), abs(p - c)
                    pred = a if (pa <= pb and pa <= pc) else (b if pb <= pc else c)
                    cur[i] = (cur[i] + pred) & 255
                else:
                    raise ValueError(f"PNG: bad filter type {ftype}")
        out[y] = cur
        prev = cur
    return out, pos


def _samples(rows, width, depth, nch):
    """Scanline bytes -> integer samples [h, width*nch] (big-endian 16-bit, packed < 8-bit)."""
    h = rows.shape[0]
    if depth == 8:
        return rows[:, :width * nch].astype(np.int64)
    if depth == 16:
        return (rows[:, 0:2 * width * nch:2].astype(np.int64) << 8) | rows[:, 1:2 * width * nch:2]
    per = 8 // depth
    bits = np.unpackbits(rows, axis=1) if depth == 1 else None
    if depth == 1:
        return bits[:, :width * nch].astype(np.int64)
    shifts = np.arange(per - 1, -1, -1) * depth
    vals = (rows[:, :, None].astype(np.int64) >> shifts) & ((1 << depth) - 1)
    return vals.reshape(h, -1)[:, :width * nch]


def read_png(path):
    with open(path, "rb") as f:
        data = f.read()
    if data[:8] != b"\x89PNG\r\n\x1a\n":
        raise ValueError(f"Error opening file: {path} (not a PNG)")
    pos, ihdr, idat, palette, trns = 8, None, [], None, None
    while pos + 8 <= len(data):
        length, tag = struct.unpack(">I4s", data[pos:pos + 8])
        body = data[pos + 8:pos + 8 + length]
        pos += 12 + length
        if tag == b"IHDR":
            ihdr = struct.unpack(">IIBBBBB", body)
        elif tag == b"PLTE":
            palette = np.frombuffer(body, np.uint8).reshape(-1, 3).astype(np.int64)
        elif tag == b"tRNS":
            trns = body
        elif tag == b"IDAT":
            idat.append(body)
        elif tag == b"CgBI":
            raise ValueError(f"{path}: Apple CgBI PNGs are not supported")
        elif tag == b"IEND":
            break
    if ihdr is None or not idat:
        raise ValueError(f"{path}: corrupt PNG")
    w, h, depth, color, comp, filt, interlace = ihdr
    if color not in _CHANNELS or comp != 0 or filt != 0 or interlace > 1:
        raise ValueError(f"{path}: unsupported PNG header")
    if depth not in (1, 2, 4, 8, 16) or (color in (2, 4, 6) and depth < 8) or (color == 3 and depth == 16):
        raise ValueError(f"{path}: bad PNG bit depth {depth} for color type {color}")
    if color == 3 and palette is None:
        raise ValueError(f"{path}: palette PNG without PLTE")
    nch = _CHANNELS[color]
    bpp = max(1, nch * depth // 8)
    buf = zlib.decompress(b"".join(idat))
    img = np.zeros((h, w * nch), np.int64)
    passes = _ADAM7 if interlace else ((0, 0, 1, 1),)
    pos = 0
    for x0, y0, dx, dy in passes:
        pw, ph = (w - x0 + dx - 1) // dx, (h - y0 + dy - 1) // dy
        if pw <= 0 or ph <= 0:
            continue
        stride = (pw * nch * depth + 7) // 8
        rows, used = _unfilter(buf[pos:], pw, ph, bpp, stride)
        pos += used
        s = _samples(rows, pw, depth, nch).reshape(ph, pw, nch)
        img.reshape(h, w, nch)[y0::dy, x0::dx] = s
    img = img.reshape(h, w, nch)
    if color == 3:
        idx = img[..., 0]
        if idx.max(initial=0) >= palette.shape[0]:
            raise ValueError(f"{path}: palette index out of range")
        img = palette[idx]
        nch = 3
    elif color == 0 and depth < 8:
        img = img * {1: 0xFF, 2: 0x55, 4: 0x11}[depth]  # stbi__depth_scale_table (:4647,4783)
    if nch >= 3:  # stbi__compute_y / _16 (alpha dropped); gray(+alpha) keeps channel 0
        gray = ((img[..., 0] * 77) + (img[..., 1] * 150) + (29 * img[..., 2])) >> 8
    else:
        gray = img[..., 0]
    if depth == 16:
        gray = (gray >> 8) & 0xFF  # 16 -> 8 bit (:1198)
    return gray.astype(np.float32) / np.float32(255.0)
