"""PNG loader: pt_png_read / pt_image_load_png against the
reference's decoding rules (src/png_decoder.cpp:40-128 driving libpng, then
src/image.cpp:60-79's byte / 255.0f):
  - 16-bit samples keep their high byte (png_set_strip_16),
  - RGB gets a filler alpha byte 0 (png_set_filler(0, PNG_FILLER_AFTER)),
  - palette images expand to RGB, and a tRNS chunk becomes alpha (entries past
    tRNS are opaque 255); without tRNS the filler 0 applies,
  - Adam7 interlacing is undone (png_read_image).
The synthetic files come from a small encoder in this test (every filter type,
both interlace modes); the expected images are computed from the source pixels
with the rules above, independently of any decoder, and PIL (present here)
cross-checks that the files are valid PNGs.  The reference's own PNG assets
(test.png, image.png, sky01/) are compared against PIL's decode when
/root/reference is mounted.  libpng itself is not available here, so parity
with it rests on these rules: "parity unpinned" against libpng's binary.
"""
import os
import struct
import zlib

import numpy as np
import pytest

import pathtrace as pt

ADAM7 = [(0, 0, 8, 8), (4, 0, 8, 8), (0, 4, 4, 8), (2, 0, 4, 4), (0, 2, 2, 4), (1, 0, 2, 2), (0, 1, 1, 2)]


def chunk(t: bytes, d: bytes, bad_crc=False) -> bytes:
    crc = zlib.crc32(t + d) & 0xFFFFFFFF
    if bad_crc:
        crc ^= 1
    return struct.pack(">I", len(d)) + t + d + struct.pack(">I", crc)


def pack_row(vals, depth):
    """vals: per-sample ints of one row (already interleaved)."""
    if depth == 8:
        return bytes(int(v) for v in vals)
    if depth == 16:
        return b"".join(struct.pack(">H", int(v)) for v in vals)
    out, acc, nb = bytearray(), 0, 0
    for v in vals:
        acc = (acc << depth) | int(v)
        nb += depth
        if nb == 8:
            out.append(acc)
            acc, nb = 0, 0
    if nb:
        out.append(acc << (8 - nb))
    return bytes(out)


def paeth(a, b, c):
    p = a + b - c
    pa, pb, pc = abs(p - a), abs(p - b), abs(p - c)
    if pa <= pb and pa <= pc:
        return a
    return b if pb <= pc else c


def filter_rows(rows, bpp, start_filter):
    out, prev = bytearray(), bytes(len(rows[0])) if rows else b""
    for k, r in enumerate(rows):
        f = (start_filter + k) % 5
        enc = bytearray()
        for i, x in enumerate(r):
            a = r[i - bpp] if i >= bpp else 0
            b = prev[i]
            c = prev[i - bpp] if i >= bpp else 0
            pred = [0, a, b, (a + b) // 2, paeth(a, b, c)][f]
            enc.append((x - pred) & 0xFF)
        out += bytes([f]) + enc
        prev = r
    return bytes(out)


def encode(samples, ctype, depth, interlace=False, plte=None, trns=None, bad_ancillary=False):
    """samples: h x w x channels int array."""
    h, w, ch = samples.shape
    bpp = max(1, ch * depth // 8)
    passes = ADAM7 if interlace else [(0, 0, 1, 1)]
    raw = b""
    for k, (x0, y0, dx, dy) in enumerate(passes):
        sub = samples[y0::dy, x0::dx]
        if sub.shape[0] == 0 or sub.shape[1] == 0:
            continue
        rows = [pack_row(sub[y].reshape(-1), depth) for y in range(sub.shape[0])]
        raw += filter_rows(rows, bpp, k)
    png = b"\x89PNG\r\n\x1a\n" + chunk(b"IHDR", struct.pack(">IIBBBBB", w, h, depth, ctype, 0, 0, int(interlace)))
    if plte is not None:
        png += chunk(b"PLTE", bytes(np.asarray(plte, dtype=np.uint8).reshape(-1)))
    if trns is not None:
        png += chunk(b"tRNS", bytes(trns), bad_crc=bad_ancillary)
    z = zlib.compress(raw, 9)
    for i in range(0, len(z), 97):  # several IDAT chunks
        png += chunk(b"IDAT", z[i:i + 97])
    return png + chunk(b"IEND", b"")


def expected(samples, ctype, depth, plte=None, trns=None):
    h, w, _ = samples.shape
    out = np.zeros((h, w, 4), dtype=np.int64)
    if ctype == 3:
        pal = np.asarray(plte, dtype=np.int64)
        out[..., :3] = pal[samples[..., 0]]
        if trns is None:
            out[..., 3] = 0
        else:
            t = np.full(256, 255, dtype=np.int64)
            t[:len(trns)] = list(trns)
            out[..., 3] = t[samples[..., 0]]
    else:
        v = samples >> 8 if depth == 16 else samples
        out[..., :samples.shape[2]] = v
        if samples.shape[2] == 3:
            out[..., 3] = 0
    return out.astype(np.float32) / np.float32(255.0)


CASES = []
for interlace in (False, True):
    for ctype, depth in [(2, 8), (6, 8), (2, 16), (6, 16)]:
        CASES.append((ctype, depth, interlace, None))
    for depth in (1, 2, 4, 8):
        CASES.append((3, depth, interlace, None))
        CASES.append((3, depth, interlace, "trns"))


@pytest.mark.parametrize("ctype,depth,interlace,trns", CASES,
                         ids=["c%d_d%d_%s%s" % (c, d, "i" if i else "p", "_trns" if t else "") for c, d, i, t in CASES])
def test_png_decode_rules(built, tmp_path, ctype, depth, interlace, trns):
    rng = np.random.default_rng(ctype * 100 + depth * 10 + int(interlace))
    h, w = 13, 11  # odd sizes: partial Adam7 passes and partial bytes at depth < 8
    plte = tr = None
    if ctype == 3:
        n = 1 << depth
        plte = rng.integers(0, 256, size=(n, 3))
        samples = rng.integers(0, n, size=(h, w, 1))
        if trns:
            tr = list(rng.integers(0, 256, size=max(1, n // 2)))  # short tRNS: later entries opaque
    else:
        ch = 3 if ctype == 2 else 4
        samples = rng.integers(0, 1 << depth, size=(h, w, ch))
    path = tmp_path / "t.png"
    path.write_bytes(encode(samples, ctype, depth, interlace, plte, tr))
    got = pt.load_png(str(path))
    want = expected(samples, ctype, depth, plte, tr)
    assert got.shape == want.shape
    assert np.array_equal(got.view(np.uint32), want.view(np.uint32))
    try:
        from PIL import Image as PILImage
    except ImportError:
        return
    im = PILImage.open(path)
    im.load()  # the file is a valid PNG by an independent decoder
    assert im.size == (w, h)


def test_png_bad_ancillary_crc_is_ignored(built, tmp_path):
    rng = np.random.default_rng(5)
    plte = rng.integers(0, 256, size=(4, 3))
    samples = rng.integers(0, 4, size=(5, 6, 1))
    p = tmp_path / "t.png"
    p.write_bytes(encode(samples, 3, 2, plte=plte, trns=[7, 9], bad_ancillary=True))
    # libpng discards an ancillary chunk with a bad CRC: no tRNS, so the filler applies
    assert np.array_equal(pt.load_png(str(p)), expected(samples, 3, 2, plte, None))


def test_png_errors(built, tmp_path):
    rng = np.random.default_rng(6)
    g = tmp_path / "g.png"
    g.write_bytes(encode(rng.integers(0, 256, size=(3, 3, 1)), 0, 8))
    with pytest.raises(pt.PtError, match="grayscale"):
        pt.load_png(str(g))
    bad = bytearray(encode(rng.integers(0, 256, size=(3, 3, 3)), 2, 8))
    bad[30] ^= 0xFF  # inside the IHDR: critical-chunk CRC error
    b = tmp_path / "b.png"
    b.write_bytes(bytes(bad))
    with pytest.raises(pt.PtError, match="CRC"):
        pt.load_png(str(b))
    n = tmp_path / "n.png"
    n.write_bytes(b"not a png at all")
    with pytest.raises(pt.PtError):
        pt.load_png(str(n))
    with pytest.raises(pt.PtError):
        pt.load_png(str(tmp_path / "missing.png"))
    trunc = tmp_path / "t.png"
    full = encode(rng.integers(0, 256, size=(40, 40, 3)), 2, 8)
    trunc.write_bytes(full[:len(full) // 2])
    with pytest.raises(pt.PtError):
        pt.load_png(str(trunc))


def test_image_dispatch_by_extension(built, tmp_path):
    rng = np.random.default_rng(7)
    samples = rng.integers(0, 256, size=(4, 5, 4))
    p = tmp_path / "x.PNG"
    p.write_bytes(encode(samples, 6, 8))
    im = pt.Image(path=str(p))
    assert np.array_equal(im.data, expected(samples, 6, 8))
    s = pt._lib.lib().pt_scene_create()
    try:
        assert pt._lib.lib().pt_image_load(s, str(p).encode()) == 0
        assert pt._lib.lib().pt_image_load_png(s, str(p).encode()) == 1
        assert pt._lib.lib().pt_image_load(s, str(tmp_path / "x.tga").encode()) < 0
    finally:
        pt._lib.lib().pt_scene_destroy(s)
    with pytest.raises(pt.PtError):
        pt.Image(path=str(tmp_path / "noext"))


GOLD = os.path.join(os.path.dirname(__file__), "golden")


def test_reference_test_png_fixture(built):
    """tests/golden/test.png is the reference's own test.png (4x3 RGB);
    png_test.npy is its decode made by make_golden.py (PIL + the rules)."""
    got = pt.load_png(os.path.join(GOLD, "test.png"))
    want = np.load(os.path.join(GOLD, "png_test.npy"))
    assert np.array_equal(got.view(np.uint32), want.view(np.uint32))


@pytest.mark.skipif(not os.path.isdir("/root/reference/sky01"), reason="reference assets not mounted")
@pytest.mark.parametrize("name", ["image.png", "sky01/top.png", "sky01/front.png"])
def test_reference_assets_match_pil(built, name):
    from PIL import Image as PILImage
    path = os.path.join("/root/reference", name)
    raw = PILImage.open(path)
    e = np.asarray(raw.convert("RGBA")).astype(np.int64)
    if raw.mode == "RGB":
        e[..., 3] = 0
    assert np.array_equal(pt.load_png(path), e.astype(np.float32) / np.float32(255.0))
