"""Scene(dict)'s source image reader against the reference's Image<1>::read
(bindings/zombie/demo/image.h:84-171, stb_image 2.28 for PNG).

Expected values are computed here from the pixels that were encoded, with the
reference's formulas: PFM rows in file order and gray = float(0.299 r + 0.587 g +
0.114 b in double) (image.h:72-76,136-147); PNG gray = int(byte)/255.0f after
stb's req_comp = 1 conversion ((77 r + 150 g + 29 b) >> 8, 16-bit >> 8, low depths
scaled by 0xff/0x55/0x11).  PNGs are written both by PIL and by a small encoder
below that exercises every scanline filter and Adam7 interlacing.
"""
import struct
import zlib

import numpy as np
import pytest

from zombie_bindings import _image

RNG = np.random.default_rng(7)


def _gray_ref(r, g, b):
    out = np.empty(np.shape(r), np.float32)
    for idx in np.ndindex(out.shape):
        # image.h:75 -- float operands promoted to double, summed left to right, stored as float
        out[idx] = np.float32(0.299 * float(np.float32(r[idx])) + 0.587 * float(np.float32(g[idx]))
                              + 0.114 * float(np.float32(b[idx])))
    return out


def _write_pfm(path, px, little=True, header=None):
    h, w = px.shape[:2]
    ch = 3 if px.ndim == 3 else 1
    hdr = header or (b"PF" if ch == 3 else b"Pf") + b"\n%d %d\n%s\n" % (w, h, b"-1.0" if little else b"1.0")
    with open(path, "wb") as f:
        f.write(hdr)
        f.write(np.ascontiguousarray(px, "<f4" if little else ">f4").tobytes())


def test_pfm_rows_in_file_order(tmp_path):
    """readPFM keeps the file's row order: buffer row 0 = the first row in the file."""
    px = RNG.standard_normal((5, 7)).astype(np.float32)
    for little in (True, False):
        path = tmp_path / f"a{int(little)}.pfm"
        _write_pfm(path, px, little)
        got = _image.read_image(str(path))
        np.testing.assert_array_equal(got, _gray_ref(px, px, px))
        assert got.dtype == np.float32 and got.shape == (5, 7)
        # rows are not mirrored: file row 0 (the minimum of a row ramp) stays row 0
    ramp = np.repeat(np.arange(4, dtype=np.float32)[:, None], 3, axis=1)
    _write_pfm(tmp_path / "r.pfm", ramp)
    assert np.all(np.diff(_image.read_image(str(tmp_path / "r.pfm"))[:, 0]) > 0)


def test_pfm_gray_in_double(tmp_path):
    """A 1-channel value is widened to (v, v, v) and re-weighted in double: the result
    is float(0.299v + 0.587v + 0.114v) (image.h:75), evaluated here pixel by pixel."""
    v = RNG.standard_normal(4096).astype(np.float32).reshape(64, 64)
    _write_pfm(tmp_path / "g.pfm", v)
    got = _image.read_image(str(tmp_path / "g.pfm"))
    ref = _gray_ref(v, v, v)
    np.testing.assert_array_equal(got, ref)


def test_pfm_rgb_and_header_tokens(tmp_path):
    px = RNG.random((3, 4, 3)).astype(np.float32)
    # operator>> tolerates extra whitespace between header tokens (image.h:113-131)
    _write_pfm(tmp_path / "c.pfm", px, header=b"PF\n  4\t3 \n-1\n")
    np.testing.assert_array_equal(_image.read_image(str(tmp_path / "c.pfm")),
                                  _gray_ref(px[..., 0], px[..., 1], px[..., 2]))


def test_unsupported_extension_and_bad_header(tmp_path):
    p = tmp_path / "x.PFM"            # hasExtension is case-sensitive (image.h:218-222)
    _write_pfm(p, np.zeros((2, 2), np.float32))
    with pytest.raises(ValueError, match="not supported"):
        _image.read_image(str(p))
    q = tmp_path / "y.pfm"
    q.write_bytes(b"QF\n1 1\n-1\n\0\0\0\0")
    with pytest.raises(ValueError, match="Invalid PFM"):
        _image.read_image(str(q))


# ------------------------------------------------------------------ PNG

def _png_bytes(raw_rows, w, h, depth, color, interlace=0, plte=None, filt=None):
    """Minimal PNG encoder: raw_rows(x0, y0, dx, dy) -> list of unfiltered scanline bytes."""
    nch = {0: 1, 2: 3, 3: 1, 4: 2, 6: 4}[color]
    bpp = max(1, nch * depth // 8)
    passes = ((0, 0, 8, 8), (4, 0, 8, 8), (0, 4, 4, 8), (2, 0, 4, 4), (0, 2, 2, 4), (1, 0, 2, 2),
              (0, 1, 1, 2)) if interlace else ((0, 0, 1, 1),)
    out = bytearray()
    k = 0
    for x0, y0, dx, dy in passes:
        rows = raw_rows(x0, y0, dx, dy)
        prev = bytes(len(rows[0])) if rows else b""
        for line in rows:
            ft = (k % 5) if filt is None else filt
            k += 1
            enc = bytearray(len(line))
            for i in range(len(line)):
                a = line[i - bpp] if i >= bpp else 0
                b = prev[i]
                c = prev[i - bpp] if i >= bpp else 0
                if ft == 0:
                    pred = 0
                elif ft == 1:
                    pred = a
                elif ft == 2:
                    pred = b
                elif ft == 3:
                    pred = (a + b) >> 1
                else:
                    p = a + b - c
                    pa, pb, pc = abs(p - a), abs(p - b), abs(p - c)
                    pred = a if (pa <= pb and pa <= pc) else (b if pb <= pc else c)
                enc[i] = (line[i] - pred) & 255
            out += bytes([ft]) + bytes(enc)
            prev = line

    def chunk(tag, data):
        return struct.pack(">I", len(data)) + tag + data + struct.pack(">I", zlib.crc32(tag + data) & 0xFFFFFFFF)

    body = chunk(b"IHDR", struct.pack(">IIBBBBB", w, h, depth, color, 0, 0, interlace))
    if plte is not None:
        body += chunk(b"PLTE", plte.astype(np.uint8).tobytes())
    return b"\x89PNG\r\n\x1a\n" + body + chunk(b"IDAT", zlib.compress(bytes(out))) + chunk(b"IEND", b"")


def _pack(samples, depth):
    """samples [n] ints -> scanline bytes at the given bit depth (big-endian 16-bit)."""
    if depth == 8:
        return bytes(np.asarray(samples, np.uint8))
    if depth == 16:
        return np.asarray(samples, ">u2").tobytes()
    per = 8 // depth
    s = list(samples) + [0] * (-len(samples) % per)
    return bytes(sum(v << (8 - depth * (j + 1)) for j, v in enumerate(s[i:i + per])) for i in range(0, len(s), per))


def _roundtrip(tmp_path, name, px, depth, color, interlace=0, plte=None):
    h, w = px.shape[:2]
    flat = px.reshape(h, w, -1)

    def rows(x0, y0, dx, dy):
        return [_pack(flat[y, x0::dx].reshape(-1), depth) for y in range(y0, h, dy) if len(range(x0, w, dx))]
    path = tmp_path / name
    path.write_bytes(_png_bytes(rows, w, h, depth, color, interlace, plte))
    return _image.read_image(str(path))


def _y(r, g, b):
    return ((r.astype(np.int64) * 77) + (g.astype(np.int64) * 150) + (29 * b.astype(np.int64))) >> 8


def _f(byte):
    return np.asarray(byte).astype(np.float32) / np.float32(255.0)


@pytest.mark.parametrize("interlace", [0, 1])
def test_png_gray8_all_filters(tmp_path, interlace):
    px = RNG.integers(0, 256, (13, 11), dtype=np.uint8)
    got = _roundtrip(tmp_path, "g.png", px, 8, 0, interlace)
    np.testing.assert_array_equal(got, _f(px))
    assert got.dtype == np.float32


@pytest.mark.parametrize("depth", [1, 2, 4])
def test_png_gray_low_depth_scaled(tmp_path, depth):
    px = RNG.integers(0, 1 << depth, (6, 19))
    got = _roundtrip(tmp_path, "l.png", px, depth, 0, 1)
    scale = {1: 0xFF, 2: 0x55, 4: 0x11}[depth]
    np.testing.assert_array_equal(got, _f(px * scale))


@pytest.mark.parametrize("interlace", [0, 1])
def test_png_rgb_rgba_gray_alpha(tmp_path, interlace):
    rgb = RNG.integers(0, 256, (9, 10, 3), dtype=np.uint8)
    np.testing.assert_array_equal(_roundtrip(tmp_path, "c.png", rgb, 8, 2, interlace),
                                  _f(_y(rgb[..., 0], rgb[..., 1], rgb[..., 2])))
    rgba = RNG.integers(0, 256, (9, 10, 4), dtype=np.uint8)
    np.testing.assert_array_equal(_roundtrip(tmp_path, "a.png", rgba, 8, 6, interlace),
                                  _f(_y(rgba[..., 0], rgba[..., 1], rgba[..., 2])))
    ga = RNG.integers(0, 256, (9, 10, 2), dtype=np.uint8)
    np.testing.assert_array_equal(_roundtrip(tmp_path, "ga.png", ga, 8, 4, interlace), _f(ga[..., 0]))


def test_png_16bit(tmp_path):
    g16 = RNG.integers(0, 65536, (5, 8))
    np.testing.assert_array_equal(_roundtrip(tmp_path, "g16.png", g16, 16, 0), _f(g16 >> 8))
    c16 = RNG.integers(0, 65536, (5, 8, 3))
    np.testing.assert_array_equal(_roundtrip(tmp_path, "c16.png", c16, 16, 2, 1),
                                  _f(_y(c16[..., 0], c16[..., 1], c16[..., 2]) >> 8))


def test_png_palette(tmp_path):
    pal = RNG.integers(0, 256, (16, 3))
    idx = RNG.integers(0, 16, (7, 9))
    for depth in (4, 8):
        got = _roundtrip(tmp_path, f"p{depth}.png", idx, depth, 3, 0, plte=pal)
        col = pal[idx]
        np.testing.assert_array_equal(got, _f(_y(col[..., 0], col[..., 1], col[..., 2])))


def test_png_written_by_pil(tmp_path):
    PIL = pytest.importorskip("PIL.Image")
    rgb = RNG.integers(0, 256, (33, 21, 3), dtype=np.uint8)
    PIL.fromarray(rgb, "RGB").save(tmp_path / "pil.png")
    np.testing.assert_array_equal(_image.read_image(str(tmp_path / "pil.png")),
                                  _f(_y(rgb[..., 0], rgb[..., 1], rgb[..., 2])))
    g = RNG.integers(0, 256, (17, 40), dtype=np.uint8)
    PIL.fromarray(g, "L").save(tmp_path / "pil_l.png", optimize=True)
    np.testing.assert_array_equal(_image.read_image(str(tmp_path / "pil_l.png")), _f(g))


def _quadrant_lookup(img, x, pmin, extent):
    """scene.h:196 uv = (x - pMin) / extent (float), image.h:54-55 row = clamp(int(v h)), col = clamp(int(u w))."""
    h, w = img.shape
    u = np.float32(np.float32(x[0] - pmin[0]) / extent[0])
    v = np.float32(np.float32(x[1] - pmin[1]) / extent[1])
    i = min(max(int(np.float32(v * np.float32(h))), 0), h - 1)
    j = min(max(int(np.float32(u * np.float32(w))), 0), w - 1)
    return img[i, j]


def quadrant_image(h=40, w=60):
    """Asymmetric test source: a different constant per quadrant of the image, in file
    order -- file row 0 is the minimum-y side of the domain in the reference's lookup."""
    img = np.empty((h, w), np.float32)
    img[:h // 2, :w // 2] = 1.0    # low y, low x
    img[:h // 2, w // 2:] = 2.0    # low y, high x
    img[h // 2:, :w // 2] = -1.0   # high y, low x
    img[h // 2:, w // 2:] = -2.0   # high y, high x
    return img


def test_scene_dict_quadrant_lookup(tmp_path):
    """The grid Scene(dict) hands to the engine, looked up as the reference's source
    callback does, returns the FILE's quadrant values (no mirroring) for PFM and PNG."""
    img = quadrant_image()
    _write_pfm(tmp_path / "q.pfm", img)
    png_px = ((img + 2.0) * 50.0).astype(np.uint8)       # 150, 200, 50, 0
    PIL = pytest.importorskip("PIL.Image")
    PIL.fromarray(png_px, "L").save(tmp_path / "q.png")
    pmin, extent = np.float32([-1.0, -0.5]), np.float32([3.0, 1.2])
    pts = {"ll": (-0.3, -0.2), "lr": (1.5, -0.2), "ul": (-0.3, 0.5), "ur": (1.5, 0.5)}
    want = {"ll": 0, "lr": 1, "ul": 2, "ur": 3}
    pfm = _image.read_image(str(tmp_path / "q.pfm"))
    png = _image.read_image(str(tmp_path / "q.png"))
    vals_pfm = [1.0, 2.0, -1.0, -2.0]
    vals_png = [150, 200, 50, 0]
    for k, x in pts.items():
        x = np.float32(x)
        assert _quadrant_lookup(pfm, x, pmin, extent) == _gray_ref(*[np.float32([vals_pfm[want[k]]])] * 3)[0]
        assert _quadrant_lookup(png, x, pmin, extent) == np.float32(vals_png[want[k]]) / np.float32(255.0)
