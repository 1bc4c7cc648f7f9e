"""User-defined Texture subclasses on the device (reference
include/texture.h:10-27: the scene API is open by the virtual getColor /
getFloat).  A caller gives the subclass's getColor (and optionally getFloat)
as device source through pt_tex_device; the scene's modules compile it in.
The same text, compiled on the host with -ffp-contract=off, is registered as
the CPU oracle's function for the texture (oracle_py.register_user_texture),
so renders and lookups are checked bit for bit.  The C++ facade's route (a
Texture subclass overriding deviceGetColor) is tests/test_facade.py's
`usertex` case."""
import ctypes
import os
import subprocess

import numpy as np
import pytest

import pathtrace as pt
from pathtrace.scene import (ColorTexture, DeviceTexture, Material, Plane, Sphere, Union, to_text)

# a 3-D checkerboard (the kind of procedural texture the reference's API invites)
CHECKER = """
    const float s = prm[0];
    const float k = floorf(p.x * s) + floorf(p.y * s) + floorf(p.z * s);
    const float odd = k - 2.0f * floorf(k * 0.5f);
    return odd != 0.0f ? mk(prm[1], prm[2], prm[3]) : mk(prm[4], prm[5], prm[6]);
"""
CHECKER_PRM = (2.0, 1.0, 0.9, 0.3, 0.2, 0.3, 1.0)
# the same body as tests/cpp/facade_p1.cpp's CheckerTexture hands the device
# (its macro, expanded and stringised: one line), so build() can precompile
# the facade binary's module too
CHECKER_FACADE = ("const float s = prm[0]; const float k = floorf(p.x * s) + floorf(p.y * s) + floorf(p.z * s); "
                  "const float odd = k - 2.0f * floorf(k * 0.5f); "
                  "return odd != 0.0f ? mk(prm[1], prm[2], prm[3]) : mk(prm[4], prm[5], prm[6]);")
# a getFloat override: a scatter coefficient that halves below y = -0.2
BANDS_COLOR = "return mk(p.y, p.y * 0.5f, 0.25f);"
BANDS_VALUE = "return p.y > -0.2f ? prm[0] : prm[0] * 0.5f;"

HOST_PRELUDE = """
#include <cmath>
struct V3 { float x, y, z; };
static inline V3 mk(float x, float y, float z) { V3 r; r.x = x; r.y = y; r.z = z; return r; }
"""


def _host_fn(name, ret, body):
    conv = "V3 p = mk(pp[0], pp[1], pp[2]);"
    if ret == "V3":
        return ("static V3 %s_body(V3 p, const float *prm) {\n%s\n}\n"
                "extern \"C\" void %s(const float *pp, const float *prm, float *out) {\n"
                "  %s V3 r = %s_body(p, prm); out[0] = r.x; out[1] = r.y; out[2] = r.z;\n}\n"
                % (name, body, name, conv, name))
    return ("static float %s_body(V3 p, const float *prm) {\n%s\n}\n"
            "extern \"C\" float %s(const float *pp, const float *prm) {\n  %s return %s_body(p, prm);\n}\n"
            % (name, body, name, conv, name))


@pytest.fixture(scope="module")
def host_fns(built, tmp_path_factory):
    """the bodies compiled on the host (-ffp-contract=off) and registered with the oracle"""
    import oracle_py as O
    d = tmp_path_factory.mktemp("usertex")
    src = HOST_PRELUDE + _host_fn("checker_color", "V3", CHECKER) + _host_fn("bands_color", "V3", BANDS_COLOR) + \
        _host_fn("bands_value", "float", BANDS_VALUE)
    (d / "ut.cpp").write_text(src)
    so = str(d / "libut.so")
    subprocess.run(["g++", "-O2", "-ffp-contract=off", "-shared", "-fPIC", str(d / "ut.cpp"), "-o", so], check=True)
    lib = ctypes.CDLL(so)
    addr = lambda f: ctypes.cast(getattr(lib, f), ctypes.c_void_p).value  # noqa: E731
    O.register_user_texture(7, addr("checker_color"))
    O.register_user_texture(8, addr("bands_color"), addr("bands_value"))
    return lib


def user_scene(scatter=0.9):
    """P0's shape with the floor's emission a user checkerboard and the diffuse
    sphere's scatter coefficient a user getFloat"""
    chk = DeviceTexture(CHECKER, CHECKER_PRM, oracle_slot=7)
    bands = DeviceTexture(BANDS_COLOR, (scatter,), value_body=BANDS_VALUE, oracle_slot=8)
    diffuse = Material(ColorTexture(0.8), bands)
    mirror = Material(ColorTexture(0.99), ColorTexture(0))
    floor = Material(ColorTexture(0), ColorTexture(0), chk)
    return Union(Union(Sphere((-1, 0, -4), .5, diffuse), Sphere((1, 0, -4), .5, mirror)),
                 Union(Sphere((0, .3, -5), .5, diffuse), Plane((0, 1, 0), .5, floor)))


def facade_user_scene(body=CHECKER):
    """tests/cpp/facade_p1.cpp `usertex`: the floor's emission its CheckerTexture"""
    diffuse = Material(ColorTexture(0.8), ColorTexture(1))
    mirror = Material(ColorTexture(0.99), ColorTexture(0))
    floor = Material(ColorTexture(0), ColorTexture(0), DeviceTexture(body, CHECKER_PRM))
    return Union(Union(Sphere((-1, 0, -4), .5, diffuse), Sphere((1, 0, -4), .5, mirror)),
                 Union(Sphere((0, .3, -5), .5, diffuse), Plane((0, 1, 0), .5, floor)))


def test_user_texture_compiles_into_the_scene_module(built):
    """the body becomes part of the render module (and of its code-object key)"""
    a = pt.DeviceScene(user_scene()).compile(4)
    assert pt.DeviceScene(user_scene(scatter=0.5)).compile(4) == a  # parameters live in P, not in the source


def test_user_texture_body_error_is_a_compile_error(built):
    bad = DeviceTexture("return nope;")
    w = Union(Sphere((-1, 0, -4), .5, Material(ColorTexture(0.8), ColorTexture(1))),
              Plane((0, 1, 0), .5, Material(ColorTexture(0), ColorTexture(0), bad)))
    with pytest.raises(pt.PtError, match="nope"):
        pt.DeviceScene(w).compile(4)


def test_user_texture_rejects_empty_body(built):
    with pytest.raises(pt.PtError, match="empty getColor body"):
        pt.DeviceScene(Plane((0, 1, 0), .5, Material(ColorTexture(0), ColorTexture(0), DeviceTexture(""))))


def test_oracle_calls_the_host_function(host_fns, tmp_path):
    import oracle_py as O
    pts = np.array([[0.1, 0.2, 0.3], [-0.6, 0.7, 1.4], [2.5, -3.5, 0.25]], np.float32)
    out = O.tex_eval(to_text(Plane((0, 1, 0), .5, Material(ColorTexture(0), ColorTexture(0), DeviceTexture(
        CHECKER, CHECKER_PRM, oracle_slot=7))), str(tmp_path)), pts)
    col = np.asarray(out).reshape(-1, len(pts), 4)  # per texture (file order), per point: r g b value
    chk = col[2]  # file order: the two ColorTextures, then the checker
    want = []
    for x, y, z in pts.astype(np.float64):
        k = np.floor(np.float32(x) * np.float32(2)) + np.floor(np.float32(y) * 2) + np.floor(np.float32(z) * 2)
        want.append((1.0, 0.9, 0.3) if int(k) % 2 else (0.2, 0.3, 1.0))
    np.testing.assert_array_equal(chk[:, :3], np.array(want, np.float32))


@pytest.mark.gpu
@pytest.mark.parametrize("order", ["fast", "reference"])
def test_user_texture_render_bitexact(host_fns, tmp_path, order):
    """the GPU frame with the user textures equals the oracle's, which calls the
    host-compiled bodies, bit for bit"""
    import oracle_py as O
    W, H, spp, depth = 48, 32, 4, 4
    root = user_scene()
    gpu = pt.render(pt.DeviceScene(root), W, H, spp, depth, order=order).reshape(-1, 3)
    ref = O.render(to_text(root, str(tmp_path)), W, H, spp, depth,
                   order=O.ORDER_FAST if order == "fast" else O.ORDER_REFERENCE)
    assert np.any(gpu != 0)
    np.testing.assert_array_equal(gpu.view(np.uint32), ref.view(np.uint32))
