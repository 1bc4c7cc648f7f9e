"""The C-ABI drop-in boundary (include/pt/pt.h) without a GPU: the library
loads and exports every declared symbol, the scene constructors validate like
the reference, host-side formats (HDR, BMP, Matrix) match the reference's
bytes, and scene modules JIT-compile for gfx950."""
import ctypes
import os
import re

import numpy as np
import pytest

import pathtrace as pt
import zoo as T
from pathtrace import _lib, scenes
from pathtrace.scene import to_text

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLD = os.path.join(ROOT, "tests", "golden")


def declared_symbols():
    syms = set()
    for h in ("pt.h",):
        text = open(os.path.join(ROOT, "include", "pt", h)).read()
        text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
        syms |= set(re.findall(r"\b(pt_[a-z0-9_]+)\s*\(", text))
    return syms


def test_exports_every_declared_symbol(built):
    syms = declared_symbols()
    assert len(syms) > 30
    L = ctypes.CDLL(_lib.LIB_PATH)
    missing = [s for s in sorted(syms) if not hasattr(L, s)]
    assert not missing, missing
    assert set(_lib.SIGNATURES) == syms, (set(_lib.SIGNATURES) ^ syms)


def test_version(built):
    assert b"gfx950" in _lib.lib().pt_version()


def test_constructor_errors(built):
    L = _lib.lib()
    s = L.pt_scene_create()
    try:
        assert L.pt_sphere(s, 0, 0, 0, 1, 7) < 0  # no such material
        assert b"material" in L.pt_last_error()
        m = L.pt_material(s, -1, -1, -1, -1, 1.0, -1)  # reference defaults
        assert m == 0
        sp = L.pt_sphere(s, 0, 0, -3, 1, m)
        assert L.pt_csg(s, 9, sp, sp) < 0
        singular = (ctypes.c_float * 12)(*([0.0] * 12))
        assert L.pt_transformed(s, singular, sp) == -2  # PT_ERR_MATH: invert() throws domain_error
        assert L.pt_set_root(s, 99) < 0
        assert L.pt_set_root(s, sp) == 0
        assert L.pt_tex_image(s, 3) < 0  # no such image
    finally:
        L.pt_scene_destroy(s)


def test_text_loader_equals_constructors(built, tmp_path):
    """pt_scene_from_text builds the same device module as the constructor calls."""
    for root, depth in [(scenes.scene_p1(), 8), (T.csg_zoo(), 6), (T.texture_zoo(), 5)]:
        ds = pt.DeviceScene(root)
        k1 = _lib.lib().pt_scene_kernel_key(ds.handle, depth)
        s = _lib.lib().pt_scene_create()
        _lib.check(_lib.lib().pt_scene_from_text(s, to_text(root, str(tmp_path)).encode()))
        k2 = _lib.lib().pt_scene_kernel_key(s, depth)
        _lib.lib().pt_scene_destroy(s)
        assert k1 and k1 == k2


def test_matrix_helpers_match_reference(built):
    z = np.load(os.path.join(GOLD, "matrix.npz"))
    for k in range(len(z["angle"])):
        rot = np.array(_lib.matrix_rotate(z["axis"][k], float(z["angle"][k])), dtype=np.float32)
        np.testing.assert_array_equal(rot.view(np.uint32), z["out"][k, 0].view(np.uint32))
        if np.isnan(z["out"][k, 1]).all():
            with pytest.raises(_lib.PtError):
                _lib.matrix_inverse(z["m"][k])
        else:
            inv = np.array(_lib.matrix_inverse(z["m"][k]), dtype=np.float32)
            np.testing.assert_array_equal(inv.view(np.uint32), z["out"][k, 1].view(np.uint32))
        cat = np.array(_lib.matrix_concat(z["m"][k], z["m2"][k]), dtype=np.float32)
        np.testing.assert_array_equal(cat.view(np.uint32), z["out"][k, 2].view(np.uint32))


def test_hdr_reader_matches_reference(built):
    img = _lib.load_hdr(os.path.join(GOLD, "image53424F01.hdr"))
    ref = np.load(os.path.join(GOLD, "hdr_decode.npz"))["rgba"]
    np.testing.assert_array_equal(img.view(np.uint32), ref.view(np.uint32))


def test_hdr_writer_round_trips_reference_file(built, tmp_path):
    """writeHDR(read(f)) == f, byte for byte (SURVEY.md s4 KAT)."""
    img = _lib.load_hdr(os.path.join(GOLD, "image53424F01.hdr"))
    out = str(tmp_path / "o.hdr")
    _lib.write_hdr(out, img[..., :3])
    assert open(out, "rb").read() == open(os.path.join(GOLD, "image53424F01.hdr"), "rb").read()


def test_hdr_writer_matches_reference_bytes(built, tmp_path):
    z = np.load(os.path.join(GOLD, "hdr_write.npz"))
    for k in range(3):
        out = str(tmp_path / ("w%d.hdr" % k))
        _lib.write_hdr(out, z["rgb%d" % k])
        assert open(out, "rb").read() == z["bytes%d" % k].tobytes()


def test_bmp_writer_format_and_tonemap(built, tmp_path):
    """24-bpp BI_RGB bottom-up BMP, bytes clamp(floor(256 c)) (src/test.cpp:1037-1059);
    against the reference's matched HDR/BMP pair (HDR mantissa quantisation: <= 3/255)."""
    rgb = _lib.load_hdr(os.path.join(GOLD, "image53424F01.hdr"))[..., :3]
    out = str(tmp_path / "o.bmp")
    _lib.write_bmp(out, rgb)
    mine = open(out, "rb").read()
    ref = open(os.path.join(GOLD, "image53424F01.bmp"), "rb").read()
    assert len(mine) == len(ref)
    assert mine[:54] == ref[:54]
    a = np.frombuffer(mine[54:], dtype=np.uint8).astype(int)
    b = np.frombuffer(ref[54:], dtype=np.uint8).astype(int)
    assert np.abs(a - b).max() <= 3
    assert np.abs(a - b).mean() < 1.0


@pytest.mark.parametrize("name", ["C1", "C2", "C3", "C5"])
def test_config_scenes_compile_for_gfx950(built, name):
    cfg = scenes.CONFIGS[name]
    key = cfg.device_scene().compile(cfg.depth)
    assert re.fullmatch(r"[0-9a-f]{16}", key)


@pytest.mark.parametrize("kw,msg", [
    (dict(width=0), "positive"), (dict(spp=0), "positive"), (dict(depth=65), "depth"),
    (dict(spp=1 << 20), "spp must be"), (dict(sample_begin=-1), "samples must lie"),
    (dict(sample_begin=(1 << 20) - 2, spp=4), "samples must lie"), (dict(order="sideways"), None),
    (dict(pixels=[0, 5, 16 * 12]), "out of range"), (dict(pixels=[-1]), "out of range"),
])
def test_render_params_are_validated_before_device_work(built, kw, msg):
    """pt_render refuses bad parameters with PT_ERR_ARG before it touches a device
    (so this runs without one): the reference would assert or misbehave"""
    import pathtrace as pt
    from pathtrace import scenes
    args = dict(width=16, height=12, spp=2, depth=4)
    args.update(kw)
    ds = pt.DeviceScene(scenes.scene_p0())
    with pytest.raises((pt.PtError, KeyError, ValueError)) as ei:
        pt.render(ds, args.pop("width"), args.pop("height"), args.pop("spp"), args.pop("depth"), **args)
    if msg:
        assert msg in str(ei.value)
