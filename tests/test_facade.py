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
    subprocess.run(["g++", "-std=c++11", "-O2", "-Wall", "-Wextra", "-Werror",
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
