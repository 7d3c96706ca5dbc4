"""Image input formats: cv::imread(GRAYSCALE / COLOR) semantics of
ofdis_read_image for PNG and Netpbm (CPU only, no GPU).

The PNG files are made here by an independent encoder (Python zlib; every filter type, Adam7, bit depths
1-16, palettes, alpha, gAMA / sRGB chunks), and the expected pixels are computed from the restated
libpng / OpenCV rules in numpy:
  * gray 1/2/4-bit expands by x255 / x85 / x17 (png_do_expand); 16-bit keeps the high byte (strip_16);
  * alpha is dropped, palettes are looked up, colour output is BGR;
  * colour -> gray: png_set_rgb_to_gray(png, 1, 0.299, 0.587) -> 15-bit weights 9797 / 19234 / 3737,
    truncating for 8 bit (r == g == b passes through), rounded for 16 bit, through libpng's 8-bit gamma
    tables (floor(255 (v/255)^g + .5)) when gAMA / sRGB make the file gamma significant;
  * Netpbm colour -> gray: OpenCV's (1868 B + 9617 G + 4899 R + 8192) >> 14.
OpenCV and libpng are not in this image, so parity with them is unpinned; known anchors: pure red
(255, 0, 0) reads as 76 through PNG (OpenCV's documented result) and as 76 through PPM.
"""
import math
import struct
import zlib

import numpy as np
import pytest

import of_dis_amd as od
from of_dis_amd import _lib

# ----------------------------------------------------------------------------- independent PNG encoder

ADAM7 = [(0, 0, 8, 8), (4, 0, 8, 8), (0, 4, 4, 8), (2, 0, 4, 4), (0, 2, 2, 4), (1, 0, 2, 2), (0, 1, 1, 2)]


def _chunk(t: bytes, d: bytes) -> bytes:
    return struct.pack(">I", len(d)) + t + d + struct.pack(">I", zlib.crc32(t + d) & 0xFFFFFFFF)


def _paeth(a, b, c):
    p = a + b - c
    pa, pb, pc = abs(p - a), abs(p - b), abs(p - c)
    return a if pa <= pb and pa <= pc else (b if pb <= pc else c)


def _pack_row(samples: np.ndarray, depth: int) -> bytes:
    s = samples.astype(np.int64).ravel()
    if depth == 16:
        return s.astype(">u2").tobytes()
    if depth == 8:
        return s.astype(np.uint8).tobytes()
    per = 8 // depth
    out = bytearray((len(s) + per - 1) // per)
    for i, v in enumerate(s):
        out[i // per] |= int(v) << (8 - depth * (i % per + 1))
    return bytes(out)


def _filter_rows(rows, bpp, rng):
    out = bytearray()
    prev = bytes(len(rows[0])) if rows else b""
    for r in rows:
        ft = int(rng.integers(0, 5))
        f = bytearray(len(r))
        for i in range(len(r)):
            a = r[i - bpp] if i >= bpp else 0
            b = prev[i]
            c = prev[i - bpp] if i >= bpp else 0
            pred = (0, a, b, (a + b) >> 1, _paeth(a, b, c))[ft]
            f[i] = (r[i] - pred) & 0xFF
        out += bytes([ft]) + f
        prev = r
    return bytes(out)


def encode_png(samples: np.ndarray, ctype: int, depth: int, interlace=False, palette=None, extra=b"", seed=0):
    """samples: [h, w, nch] integer array of raw PNG samples."""
    h, w, nch = samples.shape
    rng = np.random.default_rng(seed)
    bpp = max(1, nch * depth // 8)
    if interlace:
        raw = b""
        for x0, y0, dx, dy in ADAM7:
            sub = samples[y0::dy, x0::dx]
            if sub.shape[0] and sub.shape[1]:
                raw += _filter_rows([_pack_row(r, depth) for r in sub], bpp, rng)
    else:
        raw = _filter_rows([_pack_row(r, depth) for r in samples], bpp, rng)
    ihdr = struct.pack(">IIBBBBB", w, h, depth, ctype, 0, 0, 1 if interlace else 0)
    body = _chunk(b"IHDR", ihdr) + extra
    if palette is not None:
        body += _chunk(b"PLTE", palette.astype(np.uint8).tobytes())
    comp = zlib.compress(raw, 9)
    body += _chunk(b"IDAT", comp[: len(comp) // 2]) + _chunk(b"IDAT", comp[len(comp) // 2:])  # split IDAT
    return b"\x89PNG\r\n\x1a\n" + body + _chunk(b"IEND", b"")


# ----------------------------------------------------------------------------- expected values

RC, GC = 9797, 19234
BC = 32768 - RC - GC


def _gamma_table(g):  # png_build_8bit_table / png_gamma_8bit_correct
    if 95000 <= g <= 105000:
        return np.arange(256)
    t = np.array([math.floor(255 * math.pow(v / 255.0, g * 1e-5) + 0.5) for v in range(256)])
    t[0], t[255] = 0, 255
    return t


def _recip(a):
    return math.floor(1e10 / a + 0.5)


def expected(rgb: np.ndarray, depth16: bool, want: int, is_color: bool, gamma=0):
    """rgb: [h, w, 3] values at the stream depth (8 or 16 bit) after palette/gray expansion."""
    r, g, b = (rgb[..., k].astype(np.int64) for k in range(3))
    if want == 3:
        out = np.stack([b, g, r], -1)
        return (out >> 8 if depth16 else out).astype(np.uint8)
    if not is_color:
        gray = r
    elif depth16:
        gray = (RC * r + GC * g + BC * b + 16384) >> 15
    elif gamma and not (95000 <= gamma <= 105000):
        to1 = _gamma_table(_recip(gamma))
        from1 = _gamma_table(_recip(_recip(gamma)))
        lin = (RC * to1[r] + GC * to1[g] + BC * to1[b] + 16384) >> 15
        gray = np.where((r == g) & (r == b), r, from1[lin])
    else:
        gray = np.where((r == g) & (r == b), r, (RC * r + GC * g + BC * b) >> 15)
    return ((gray >> 8) if depth16 else gray).astype(np.uint8)[..., None]


def read(path, want):
    return od.read_image(str(path), want)


# ----------------------------------------------------------------------------- tests

@pytest.mark.parametrize("interlace", [False, True])
@pytest.mark.parametrize("depth", [1, 2, 4, 8, 16])
@pytest.mark.parametrize("alpha", [False, True])
def test_png_gray(tmp_path, depth, interlace, alpha):
    if alpha and depth < 8:
        pytest.skip("gray+alpha exists at 8 and 16 bit only")
    rng = np.random.default_rng(depth)
    h, w = 13, 11
    v = rng.integers(0, 1 << depth, (h, w))
    samples = np.stack([v, rng.integers(0, 1 << depth, (h, w))], -1) if alpha else v[..., None]
    path = tmp_path / "g.png"
    path.write_bytes(encode_png(samples, 4 if alpha else 0, depth, interlace, seed=depth))
    ex = v * {1: 255, 2: 0x55, 4: 0x11, 8: 1, 16: 1}[depth]
    rgb = np.stack([ex] * 3, -1)
    for want in (1, 3):
        got = read(path, want)
        assert np.array_equal(got, expected(rgb, depth == 16, want, False)), (depth, want)


@pytest.mark.parametrize("interlace", [False, True])
@pytest.mark.parametrize("depth", [8, 16])
@pytest.mark.parametrize("alpha", [False, True])
def test_png_rgb(tmp_path, depth, interlace, alpha):
    rng = np.random.default_rng(100 + depth)
    h, w = 17, 9
    rgb = rng.integers(0, 1 << depth, (h, w, 3))
    rgb[0, :3] = rgb[0, :3, :1]  # some r == g == b pixels
    samples = np.concatenate([rgb, rng.integers(0, 1 << depth, (h, w, 1))], -1) if alpha else rgb
    path = tmp_path / "c.png"
    path.write_bytes(encode_png(samples, 6 if alpha else 2, depth, interlace, seed=depth + 7))
    for want in (1, 3):
        assert np.array_equal(read(path, want), expected(rgb, depth == 16, want, True)), (depth, want)


@pytest.mark.parametrize("depth", [1, 2, 4, 8])
def test_png_palette(tmp_path, depth):
    rng = np.random.default_rng(200 + depth)
    h, w = 10, 15
    n = 1 << depth
    pal = rng.integers(0, 256, (n, 3))
    idx = rng.integers(0, n, (h, w))
    path = tmp_path / "p.png"
    trns = _chunk(b"tRNS", bytes(range(n)))  # stripped with the alpha channel it expands to
    path.write_bytes(encode_png(idx[..., None], 3, depth, palette=pal, extra=b"", seed=depth))
    rgb = pal[idx]
    for want in (1, 3):
        assert np.array_equal(read(path, want), expected(rgb, False, want, True))
    # tRNS must come after PLTE: rebuild with it inserted before IDAT
    data = encode_png(idx[..., None], 3, depth, palette=pal, seed=depth)
    k = data.index(b"IDAT") - 4
    path.write_bytes(data[:k] + trns + data[k:])
    for want in (1, 3):
        assert np.array_equal(read(path, want), expected(rgb, False, want, True))


@pytest.mark.parametrize("chunk", ["gAMA", "sRGB", "gAMA1"])
def test_png_gamma_rgb_to_gray(tmp_path, chunk):
    rng = np.random.default_rng(7)
    rgb = rng.integers(0, 256, (12, 12, 3))
    if chunk == "gAMA":
        extra, g = _chunk(b"gAMA", struct.pack(">I", 45455)), 45455
    elif chunk == "sRGB":
        extra, g = _chunk(b"sRGB", b"\x00"), 45455
    else:  # gamma 1.0: not significant, the truncating path
        extra, g = _chunk(b"gAMA", struct.pack(">I", 100000)), 100000
    path = tmp_path / "gm.png"
    path.write_bytes(encode_png(rgb, 2, 8, extra=extra))
    assert np.array_equal(read(path, 1), expected(rgb, False, 1, True, gamma=g))
    assert np.array_equal(read(path, 3), expected(rgb, False, 3, True))  # colour output: no gamma


def test_png_known_anchors(tmp_path):
    rgb = np.array([[[255, 0, 0], [0, 255, 0], [0, 0, 255], [128, 128, 128], [255, 255, 255]]])
    path = tmp_path / "k.png"
    path.write_bytes(encode_png(rgb, 2, 8))
    assert read(path, 1)[0, :, 0].tolist() == [76, 149, 29, 128, 255]
    assert read(path, 3)[0, 0].tolist() == [0, 0, 255]  # BGR


def test_png_errors(tmp_path):
    good = encode_png(np.zeros((4, 4, 1), np.int64), 0, 8)
    bad = bytearray(good)
    bad[good.index(b"IDAT") + 6] ^= 0xFF  # corrupt the first IDAT payload byte: CRC mismatch
    (tmp_path / "bad.png").write_bytes(bytes(bad))
    (tmp_path / "trunc.png").write_bytes(good[:-20])
    (tmp_path / "x.jpg").write_bytes(b"\xff\xd8\xff\xe0" + bytes(64))
    w, h = od.lib(), None
    for name, code in (("bad.png", _lib.ERR_IO), ("trunc.png", _lib.ERR_IO), ("x.jpg", _lib.ERR_UNSUPPORTED),
                       ("missing.png", _lib.ERR_IO)):
        with pytest.raises(od.OfdisError) as e:
            read(tmp_path / name, 1)
        assert e.value.code == code, name


def test_oversized_headers_fail_cleanly(tmp_path):
    """A tiny file whose header claims a huge image is refused before any buffer is sized from it
    (OpenCV's CV_IO_MAX_IMAGE_PIXELS = 2^30), with a status code instead of an abort."""
    import zlib as _z
    for w, h in ((1 << 24, 1 << 24), (40000, 40000), (1 << 16, 1 << 15)):
        ihdr = struct.pack(">IIBBBBB", w, h, 8, 0, 0, 0, 0)
        png = b"\x89PNG\r\n\x1a\n" + _chunk(b"IHDR", ihdr) + _chunk(b"IDAT", _z.compress(b"\0" * 64)) + \
            _chunk(b"IEND", b"")
        (tmp_path / "huge.png").write_bytes(png)
        with pytest.raises(od.OfdisError) as e:
            read(tmp_path / "huge.png", 1)
        assert e.value.code == _lib.ERR_IO, (w, h)
    (tmp_path / "huge.pgm").write_bytes(b"P5\n40000 40000\n255\n" + bytes(16))
    with pytest.raises(od.OfdisError) as e:
        read(tmp_path / "huge.pgm", 1)
    assert e.value.code == _lib.ERR_IO


@pytest.mark.parametrize("kind", ["P2", "P3", "P5", "P6", "P1", "P4"])
@pytest.mark.parametrize("want", [1, 3])
def test_pnm(tmp_path, kind, want):
    rng = np.random.default_rng(ord(kind[1]))
    h, w = 6, 13
    if kind in ("P1", "P4"):
        bits = rng.integers(0, 2, (h, w))
        gray = np.where(bits == 1, 0, 255)
        if kind == "P1":
            body = "\n".join("".join(str(b) for b in row) for row in bits).encode()  # unseparated digits
        else:
            body = np.packbits(bits.astype(np.uint8), axis=1).tobytes()
        data = f"{kind}\n# comment\n{w} {h}\n".encode() + body
        rgb = np.stack([gray] * 3, -1)
        color = False
    else:
        color = kind in ("P3", "P6")
        v = rng.integers(0, 256, (h, w, 3 if color else 1))
        head = f"{kind}\n# comment\n{w} {h}\n255\n".encode()
        if kind in ("P2", "P3"):
            data = head + " ".join(str(int(x)) for x in v.ravel()).encode()
        else:
            data = head + v.astype(np.uint8).tobytes()
        rgb = v if color else np.concatenate([v] * 3, -1)
    path = tmp_path / "i.pnm"
    path.write_bytes(data)
    got = read(path, want)
    r, g, b = (rgb[..., k].astype(np.int64) for k in range(3))
    if want == 3:
        ex = np.stack([b, g, r], -1)
    elif color:
        ex = ((1868 * b + 9617 * g + 4899 * r + 8192) >> 14)[..., None]
    else:
        ex = r[..., None]
    assert np.array_equal(got, ex.astype(np.uint8))


def test_pnm_red_anchor_and_16bit(tmp_path):
    (tmp_path / "r.ppm").write_bytes(b"P6\n1 1\n255\n\xff\x00\x00")
    assert read(tmp_path / "r.ppm", 1).item() == 76
    v = np.array([[0x1234, 0xFFFF, 0x00FF]], ">u2")
    (tmp_path / "w.pgm").write_bytes(b"P5\n3 1\n65535\n" + v.tobytes())
    assert read(tmp_path / "w.pgm", 1)[0, :, 0].tolist() == [0x12, 0xFF, 0x00]


# ----------------------------------------------------------------------------- BMP (OpenCV BmpDecoder semantics)

def encode_bmp(kind, bgr, idx=None, palette=None, top_down=False, header=40):
    """An independent BMP writer: kind in pal1/pal4/pal8 (idx [h][w], palette [n][3] BGR), 555, 565, 24, 32
    (bgr [h][w][3], low bits ignored by the 16-bit packing); header 40 (INFO), 124 (V5) or 12 (CORE)."""
    h, w = (idx if idx is not None else bgr).shape[:2]
    bpp = {"pal1": 1, "pal4": 4, "pal8": 8, "555": 16, "565": 16, "24": 24, "32": 32}[kind]
    stride = ((w * bpp + 31) // 32) * 4
    rows = []
    for y in range(h):
        if kind.startswith("pal"):
            vals = idx[y].astype(np.uint8)
            if bpp == 8:
                r = vals.tobytes()
            elif bpp == 4:
                v = np.concatenate([vals, np.zeros(len(vals) % 2, np.uint8)])
                r = ((v[0::2] << 4) | v[1::2]).astype(np.uint8).tobytes()
            else:
                r = np.packbits(vals.astype(np.uint8)).tobytes()
        elif kind in ("555", "565"):
            b, g, rr = (bgr[y, :, k].astype(np.uint16) for k in range(3))
            t = (b >> 3) | ((g >> 3) << 5) | ((rr >> 3) << 10) if kind == "555" else (b >> 3) | ((g >> 2) << 5) | ((rr >> 3) << 11)
            r = t.astype("<u2").tobytes()
        elif kind == "24":
            r = bgr[y].astype(np.uint8).tobytes()
        else:
            r = np.concatenate([bgr[y], np.full((w, 1), 7, np.uint8)], 1).astype(np.uint8).tobytes()
        rows.append(r + b"\0" * (stride - len(r)))
    if not top_down:
        rows = rows[::-1]
    pix = b"".join(rows)
    comp = 3 if kind == "565" else 0
    masks = struct.pack("<III", 0xF800, 0x07E0, 0x001F) if kind == "565" else b""
    pal = b""
    if kind.startswith("pal"):
        ent = 3 if header == 12 else 4
        pal = b"".join(bytes(list(c)) + (b"" if ent == 3 else b"\0") for c in palette)
    if header == 12:
        dib = struct.pack("<IHHHH", 12, w, h, 1, bpp)
    else:
        dib = struct.pack("<IiiHHIIiiII", header, w, -h if top_down else h, 1, bpp, comp, len(pix), 2835, 2835,
                          len(palette) if palette is not None else 0, 0)
        if header > 40:
            dib += (masks + b"\0" * (header - 40))[: header - 40]
            masks = b""
    off = 14 + len(dib) + len(masks) + len(pal)
    return b"BM" + struct.pack("<IHHI", off + len(pix), 0, 0, off) + dib + masks + pal + pix


@pytest.mark.parametrize("kind", ["pal1", "pal4", "pal8", "555", "565", "24", "32"])
@pytest.mark.parametrize("top_down,header", [(False, 40), (True, 40), (False, 124), (False, 12)])
@pytest.mark.parametrize("want", [1, 3])
def test_bmp(tmp_path, kind, top_down, header, want):
    if header == 12 and (kind in ("555", "565", "32") or top_down):
        pytest.skip("OS/2 core headers: palette and 24-bit images, bottom-up")
    rng = np.random.default_rng(len(kind) + header)
    h, w = 7, 13
    idx = palette = None
    if kind.startswith("pal"):
        n = {"pal1": 2, "pal4": 16, "pal8": 256}[kind]
        palette = rng.integers(0, 256, (n, 3))
        idx = rng.integers(0, n, (h, w))
        bgr = palette[idx]
    else:
        bgr = rng.integers(0, 256, (h, w, 3))
        if kind == "555":
            bgr = bgr & 0xF8
        elif kind == "565":
            bgr = bgr & np.array([0xF8, 0xFC, 0xF8])
    path = tmp_path / "i.bmp"
    path.write_bytes(encode_bmp(kind, bgr, idx, palette, top_down, header))
    got = read(path, want)
    b, g, r = (bgr[..., k].astype(np.int64) for k in range(3))
    ex = np.stack([b, g, r], -1) if want == 3 else ((1868 * b + 9617 * g + 4899 * r + 8192) >> 14)[..., None]
    assert np.array_equal(got, ex.astype(np.uint8)), (kind, top_down, header, want)


def test_bmp_refused_forms(tmp_path):
    bgr = np.zeros((2, 3, 3), np.uint8)
    data = bytearray(encode_bmp("24", bgr))
    data[30:34] = struct.pack("<I", 1)  # BI_RLE8
    (tmp_path / "rle.bmp").write_bytes(bytes(data))
    with pytest.raises(_lib.OfdisError) as e:
        read(tmp_path / "rle.bmp", 3)
    assert e.value.code == _lib.ERR_UNSUPPORTED
    (tmp_path / "short.bmp").write_bytes(encode_bmp("24", bgr)[:-5])
    with pytest.raises(_lib.OfdisError) as e:
        read(tmp_path / "short.bmp", 3)
    assert e.value.code == _lib.ERR_IO
