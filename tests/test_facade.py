"""The C++ host facade (include/pt/PathTrace.hpp): reference-style scene code
(tests/cpp/facade_p1.cpp builds P1 with `new Sphere(...)`, `Material`, ...)
compiles with g++ against the facade + libpt.so, maps errors to the
reference's exception types, and flattens to the same device scene as the
Python mirror.  The GPU case renders through it and compares bit for bit."""
import os
import subprocess

import numpy as np
import pytest

import pathtrace as pt
from pathtrace import scenes

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIBDIR = os.path.join(ROOT, "path-trace_amd", "lib")


@pytest.fixture(scope="module")
def facade_bin(built, tmp_path_factory):
    out = str(tmp_path_factory.mktemp("facade") / "facade_p1")
    subprocess.run(["g++", "-std=c++11", "-O2", "-Wall", "-Wextra", "-Werror", "-pthread",
                    "-I" + os.path.join(ROOT, "include"), os.path.join(ROOT, "tests", "cpp", "facade_p1.cpp"),
                    "-L" + LIBDIR, "-lpt", "-Wl,-rpath," + LIBDIR, "-o", out], check=True)
    return out


def test_facade_error_mapping(facade_bin):
    r = subprocess.run([facade_bin, "errors"], capture_output=True, text=True, timeout=60)
    assert r.returncode == 0, r.stderr
    assert r.stdout.startswith("errors ok")


def test_facade_flattens_like_python_mirror(facade_bin):
    r = subprocess.run([facade_bin, "key", "8"], capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr
    assert r.stdout.strip() == pt.DeviceScene(scenes.scene_p1()).compile(8)


@pytest.mark.gpu
def test_facade_render_bitexact(facade_bin, tmp_path):
    W, H, spp, depth = 40, 24, 4, 8
    out = str(tmp_path / "img.bin")
    r = subprocess.run([facade_bin, "render", str(W), str(H), str(spp), str(depth), out],
                       capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr
    got = np.fromfile(out, dtype=np.float32).reshape(-1, 3)
    want = pt.render(scenes.scene_p1(), W, H, spp, depth).reshape(-1, 3)
    np.testing.assert_array_equal(got.view(np.uint32), want.view(np.uint32))


@pytest.mark.gpu
def test_facade_trace_pixel_bitexact(facade_bin, tmp_path):
    """tracePixel(*spanIterator, x, y, W, H, spp, depth, sw, sh, dist, engine) per
    pixel -- the reference demo's call (src/test.cpp:450) against the facade --
    gives Renderer::render's frame bit for bit (same run seed, fast order).
    The binary also checks the other two overloads (exit codes 15-17): the
    engine-less one gives Renderer::render's pixel (the global FrameEngine),
    and a reference-style engine T seeds the call with two of its draws --
    the bits of a FrameEngine with that seed -- and successive calls advance
    it (fresh streams, as the reference's shared engine gives)."""
    W, H, spp, depth = 24, 16, 4, 8
    out = str(tmp_path / "tp.bin")
    r = subprocess.run([facade_bin, "tracepixel", str(W), str(H), str(spp), str(depth), out],
                       capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr
    got = np.fromfile(out, dtype=np.float32).reshape(-1, 3)
    want = pt.render(scenes.scene_p1(), W, H, spp, depth).reshape(-1, 3)
    np.testing.assert_array_equal(got.view(np.uint32), want.view(np.uint32))


@pytest.mark.gpu
def test_facade_span_iterator_matches_oracle(facade_bin, tmp_path):
    """world->makeSpanIterator() through the facade (pt_query_spans): init(Ray)
    / isAtEnd / operator* / next give the reference's span lists, bit for bit
    against the oracle (which tests/test_oracle_golden.py pins to the reference)."""
    import oracle_py as O
    import zoo as T
    from pathtrace.scene import to_text
    rays = T.random_rays(64, seed=5)
    rp, out = str(tmp_path / "rays.bin"), str(tmp_path / "spans.bin")
    rays.tofile(rp)
    r = subprocess.run([facade_bin, "spans", rp, out], capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr
    want = O.spans(to_text(scenes.scene_p1(), str(tmp_path)), rays)
    buf = open(out, "rb").read()
    pos, matmap = 0, {}
    for spans in want:
        c = int(np.frombuffer(buf, dtype=np.int32, count=1, offset=pos)[0])
        pos += 4
        assert c == len(spans)
        for (a, m0, b, m1) in spans:
            rec = np.frombuffer(buf, dtype=np.float32, count=10, offset=pos)
            pos += 40
            np.testing.assert_array_equal(rec[[0, 1, 2, 3, 5, 6, 7, 8]].view(np.uint32),
                                          np.concatenate([a, b]).view(np.uint32))
            for mine, theirs in ((rec[4:5].view(np.int32)[0], m0), (rec[9:10].view(np.int32)[0], m1)):
                assert matmap.setdefault(int(mine), theirs) == theirs  # one Material per material id
    assert pos == len(buf)


@pytest.mark.gpu
def test_facade_texture_virtuals(facade_bin, tmp_path):
    """Texture::getColor / getFloat through the facade (pt_tex_eval) for a
    mirror-ball sky map of the reference's test2.hdr, against the oracle; and a
    reference-style user subclass that overrides getColor only (host-side,
    getFloat = the reference's default mean)."""
    import oracle_py as O
    import zoo as T
    from pathtrace.scene import (ColorTexture, Image, ImageTexture, Material, MirrorBallSkymapTexture, Sphere,
                                 to_text)
    hdr = os.path.join(ROOT, "assets", "test2.hdr")
    pts = T.texture_points(256, seed=4)
    pp, out = str(tmp_path / "pts.bin"), str(tmp_path / "tex.bin")
    pts.tofile(pp)
    r = subprocess.run([facade_bin, "tex", hdr, pp, out], capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr
    got = np.fromfile(out, dtype=np.float32).reshape(-1, 8)
    scene = Sphere((0, 0, -4), 1, Material(ColorTexture(0), ColorTexture(0),
                                          MirrorBallSkymapTexture(ImageTexture(Image(path=hdr)))))
    txt = to_text(scene, str(tmp_path))
    kinds = [ln.split()[2] for ln in txt.splitlines() if ln.startswith("tex ")]
    want = O.tex_eval(txt, pts)[kinds.index("mirrorball")]
    np.testing.assert_array_equal(got[:, :4].view(np.uint32), want.view(np.uint32))
    chk = np.where((np.floor(pts).astype(np.int64).sum(axis=1) % 2) != 0, 1.0, 0.25).astype(np.float32)
    np.testing.assert_array_equal(got[:, 4], chk)
    np.testing.assert_array_equal(got[:, 7], ((chk + chk) + chk) * np.float32(1.0 / 3.0))


@pytest.mark.gpu
def test_facade_trace_ray_bitexact(facade_bin, tmp_path):
    """traceRay<T> / traceRays through the facade (pt_trace_rays): the fixture
    rays in reference order give the unmodified reference's traceRay means bit
    for bit (tests/golden/trace_p1.npz); the binary itself checks the per-call
    overload, the T-engine overload and the float-coordinate tracePixel against
    batches with the same engine keys (exit codes 10-13)."""
    d = np.load(os.path.join(ROOT, "tests", "golden", "trace_p1.npz"))
    spp, depth, _ = [int(v) for v in d["meta"]]
    rp, out = str(tmp_path / "rays.bin"), str(tmp_path / "tr.bin")
    d["rays"].astype(np.float32).tofile(rp)
    r = subprocess.run([facade_bin, "traceray", rp, str(depth), str(spp), out], capture_output=True, text=True,
                       timeout=600)
    assert r.returncode == 0, (r.returncode, r.stderr)
    got = np.fromfile(out, dtype=np.float32).reshape(-1, 3)
    np.testing.assert_array_equal(got.view(np.uint32), d["mean"].view(np.uint32))


@pytest.mark.gpu
def test_facade_pixel_batcher(facade_bin, tmp_path):
    """The demo's per-pixel call shape from 8 host threads through PixelBatcher:
    the same bits as one batch for the frame (exit code 14 otherwise), in far
    fewer launches than pixels; per-call latency recorded."""
    import json
    out = str(tmp_path / "lat.json")
    r = subprocess.run([facade_bin, "latency", "48", "32", "4", "8", "8", out], capture_output=True, text=True,
                       timeout=600)
    assert r.returncode == 0, (r.returncode, r.stderr)
    d = json.load(open(out))
    assert d["per_call_us"] > 0 and d["batcher_launches"] >= 1
    assert d["batcher_launches"] < 48 * 32 / 2
    bd = d["per_call_breakdown_us"]  # pt_call_profile: the phases of one call add up to it
    for k, ph in bd.items():
        parts = ph["setup"] + ph["enqueue"] + ph["wait"] + ph["d2h"]
        assert 0 < parts <= ph["total"] * 1.001 + 1, (k, ph)
        if k.startswith("events"):
            assert ph["kernel"] > 0 and ph["reduce"] > 0, (k, ph)


@pytest.mark.gpu
def test_facade_user_texture_bitexact(facade_bin, tmp_path):
    """A C++ Texture subclass with a host getColor override and the same body
    as deviceGetColor: the device lookups equal the host override bit for bit
    (checked in the binary, exit 18), and the frame equals the Python mirror's
    render of the same scene (pathtrace.DeviceTexture with the same text)."""
    from test_user_texture import facade_user_scene
    W, H, spp, depth = 40, 24, 4, 6
    out = str(tmp_path / "img.bin")
    r = subprocess.run([facade_bin, "usertex", str(W), str(H), str(spp), str(depth), out],
                       capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, (r.returncode, r.stderr)
    got = np.fromfile(out, dtype=np.float32).reshape(-1, 3)
    want = pt.render(facade_user_scene(), W, H, spp, depth).reshape(-1, 3)
    np.testing.assert_array_equal(got.view(np.uint32), want.view(np.uint32))


@pytest.mark.gpu
def test_facade_user_object_bitexact(facade_bin, tmp_path):
    """A C++ Object subclass whose device form is the reference sphere's
    arithmetic (deviceSpan / deviceNormal, pt_object_device), put in place of
    one of P1's spheres: the frame is P1's bit for bit."""
    W, H, spp, depth = 40, 24, 4, 8
    out = str(tmp_path / "img.bin")
    r = subprocess.run([facade_bin, "userobj", str(W), str(H), str(spp), str(depth), out],
                       capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, (r.returncode, r.stderr)
    got = np.fromfile(out, dtype=np.float32).reshape(-1, 3)
    want = pt.render(scenes.scene_p1(), W, H, spp, depth).reshape(-1, 3)
    np.testing.assert_array_equal(got.view(np.uint32), want.view(np.uint32))
