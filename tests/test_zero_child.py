"""Mirror children of weight +-0 (pt_device.h zero_child, PT_ZERO_CHILD).

A surface with reflectance 0 and no scatter loop -- a sky or an emitter --
still spawns its one mirror child in the reference (path-trace.h:137-162),
and that child's traceRay runs a query before it returns the emission where
it lands (:97-108), which the parent then adds times a weight of +-0 (:162).
The kernel skips that query when the sum cannot change: every emission in
the scene finite (codegen color_bound), the partial sum neither -0 nor NaN.
These tests render scenes inside an emissive sky sphere, so every mirror
child of the sky lands on the sky again, against the oracle (which runs every
query), bit for bit and with the same query counts:

* a finite sky: the skip is taken (wave spine, lane front end, lane walks;
  a clear glass sphere with reflectance 0 takes the lane walk's deferred
  form, mode 3, after its refraction child);
* a sky with an infinite emission channel, and one whose MultiplyTexture
  overflows to infinity: the reference's 0 * inf is NaN, so the skip must not
  be taken -- codegen marks these scenes not emis_finite.
"""
import numpy as np
import pytest

import pathtrace as pt
from pathtrace.scene import ColorTexture, Material, MultiplyTexture, Sphere, Union, to_text

INF = float("inf")


def sky_scene(emission):
    diffuse = Material(ColorTexture(0.8), ColorTexture(1))
    mirror = Material(ColorTexture(0.99), ColorTexture(0))
    # transmits, reflectance 0: its mirror child has weight +-0 once the refraction child is summed
    clear = Material(ColorTexture(0), ColorTexture(0), ColorTexture(0), ColorTexture(0.9), 1.3, ColorTexture(1))
    sky = Material(ColorTexture(0), ColorTexture(0), emission)
    return Union(Union(Sphere((-1, 0, -4), .5, diffuse), Sphere((1, 0, -4), .5, mirror)),
                 Union(Sphere((0, .3, -5), .5, clear), Sphere((0, 0, -4), 20, sky)))


SKIES = {
    "finite": lambda: ColorTexture((0.5, 0.7, 1.0)),
    "inf": lambda: ColorTexture((INF, 0.7, 1.0)),
    "overflow": lambda: MultiplyTexture((1e30, 1.0, 1.0), ColorTexture((1e20, 0.7, 1.0))),
}
# (sky, lane_walk) of the GPU cases (tests/precompile_modules.py builds their modules)
CASES = [("finite", 0), ("inf", 0), ("overflow", 0), ("finite", 2), ("inf", 2)]
W, H, SPP, DEPTH = 40, 24, 4, 5


@pytest.mark.gpu
@pytest.mark.parametrize("order", ["fast", "reference"])
@pytest.mark.parametrize("sky,lane_walk", CASES)
def test_zero_weight_children_bitexact(built, tmp_path, sky, lane_walk, order):
    import oracle_py as O
    root = sky_scene(SKIES[sky]())
    ds = pt.DeviceScene(root, lane_walk=lane_walk)
    gpu, st = pt.render(ds, W, H, SPP, DEPTH, order=order, stats=True)
    ref, rst = O.render(to_text(root, str(tmp_path)), W, H, SPP, DEPTH,
                        order=O.ORDER_FAST if order == "fast" else O.ORDER_REFERENCE, stats=True)
    gpu = gpu.reshape(-1, 3)
    np.testing.assert_array_equal(gpu.view(np.uint32), ref.view(np.uint32))
    assert st["queries"] == rst["queries"], (st["queries"], rst["queries"])
    if sky == "finite":
        assert np.all(np.isfinite(gpu)) and np.any(gpu > 0)
    else:  # the sky's mirror children make 0 * inf = NaN in the red channel
        assert np.isnan(gpu[:, 0]).any()


def test_emis_finite_is_decided_by_the_bound(built):
    """codegen's emis_finite is part of the module source: the same tree with
    other finite emissions keeps its key, an infinite channel or a product past
    FLT_MAX changes it"""
    key = lambda sky: pt.DeviceScene(sky_scene(sky)).kernel_key(DEPTH)  # noqa: E731
    finite = key(SKIES["finite"]())
    assert key(ColorTexture((2.0, 3.0, 4.0))) == finite
    assert key(SKIES["inf"]()) != finite
    assert key(ColorTexture((float("nan"), 1.0, 1.0))) == key(SKIES["inf"]())
    assert key(SKIES["overflow"]()) != key(MultiplyTexture((2.0, 1.0, 1.0), ColorTexture((1e20, 0.7, 1.0))))


def test_emis_finite_scans_image_texels(built):
    """an image-mapped emission is bounded by its texels (the lookups are
    bounds-checked): a finite image keeps the skip, one infinite texel drops it,
    and a LogTexture over that image (its filter maps +inf to +inf) too"""
    from pathtrace.scene import Image, ImageTexture, LogTexture, SphericalCoordinatesSkymapTexture
    img = np.full((8, 16, 4), 0.5, np.float32)
    bad = img.copy()
    bad[3, 5, 1] = np.inf
    key = lambda tex: pt.DeviceScene(sky_scene(tex)).kernel_key(DEPTH)  # noqa: E731
    fin = key(SphericalCoordinatesSkymapTexture(ImageTexture(Image(img))))
    inf = key(SphericalCoordinatesSkymapTexture(ImageTexture(Image(bad))))
    assert fin != inf
    assert key(SphericalCoordinatesSkymapTexture(ImageTexture(Image(img * 2)))) == fin
    assert key(LogTexture(ImageTexture(Image(bad)))) != key(LogTexture(ImageTexture(Image(img))))
