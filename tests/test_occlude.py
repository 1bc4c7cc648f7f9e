"""Leaf children occluded by a plane (pt_device.h Occl, PT_OCCLUDE).

In a tree of Unions, spheres and planes, a burst's leaf child that enters a
non-emissive plane's solid before any emissive primitive's span can start has
a non-emissive first hit or none, so its term is zero and the generation round
settles it like a dark child.  zoo.occlude_box puts the emitters close (a box
of emissive half-spaces at distance 3), so entries into the ground plane land
on both sides of the bound and its margins, with diffuse and glossy bursts
(the glossy one's |w| bound is 1 + |kR|).  The GPU frame is checked against
the oracle bit for bit with equal query counts; the build without the test
(PT_OCCLUDE=0) gives the same bits with fewer dark children.  Variants: an
emissive sphere (no bound: no claim) and a tilted ground (not axis-aligned:
no claim).
"""
import numpy as np
import pytest

import pathtrace as pt
import zoo
from pathtrace.scene import to_text

VARIANTS = ["box", "emissive_sphere", "tilted"]
W, H, SPP, DEPTH = 48, 32, 4, 3


@pytest.mark.gpu
@pytest.mark.parametrize("variant", VARIANTS)
def test_occluded_children_bitexact(built, tmp_path, variant):
    import oracle_py as O
    root = zoo.occlude_box(variant)
    gpu, st = pt.render(pt.DeviceScene(root), W, H, SPP, DEPTH, stats=True)
    ref, rst = O.render(to_text(root, str(tmp_path)), W, H, SPP, DEPTH, order=O.ORDER_FAST, stats=True)
    gpu = gpu.reshape(-1, 3)
    np.testing.assert_array_equal(gpu.view(np.uint32), ref.view(np.uint32))
    assert st["queries"] == rst["queries"], (st["queries"], rst["queries"])
    assert np.all(np.isfinite(gpu)) and np.any(gpu > 0)


@pytest.mark.gpu
def test_occlusion_settles_more_children(built, monkeypatch):
    """the occluder test is exercised: without it (PT_OCCLUDE=0, a module
    build() precompiles) the frame is the same and fewer children are dark"""
    root = zoo.occlude_box()
    on, st_on = pt.render(pt.DeviceScene(root), W, H, SPP, DEPTH, stats=True)
    monkeypatch.setenv("PT_DEVICE_DEFINES", "PT_OCCLUDE=0")
    off, st_off = pt.render(pt.DeviceScene(root), W, H, SPP, DEPTH, stats=True)
    np.testing.assert_array_equal(on.view(np.uint32), off.view(np.uint32))
    assert st_on["queries"] == st_off["queries"]
    assert st_on["dark_queries"] > st_off["dark_queries"], (st_on["dark_queries"], st_off["dark_queries"])


def test_occlude_scenes_render_on_the_oracle(built, tmp_path):
    """the scenes are well formed and lit (CPU: the oracle alone)"""
    import oracle_py as O
    for v in VARIANTS:
        img = O.render(to_text(zoo.occlude_box(v), str(tmp_path)), 16, 8, 2, DEPTH, order=O.ORDER_FAST)
        assert np.all(np.isfinite(img)) and np.any(img > 0), v
