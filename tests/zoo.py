"""Test scenes beyond the benchmark configs: every CSG operator, transformed
objects, the Difference quirk, glossy/glass/mirror materials and every texture
class of the reference (include/texture.h, image_texture.h, filter_texture.h,
transform_texture.h).  Shared by tests/golden/make_golden.py (which freezes the
reference's outputs) and the tests that compare against them."""
import math

import numpy as np

from pathtrace.scene import (ColorTexture, CoordTexture, Difference, Image, ImageAlphaTexture,
                             ImageSkyboxAlphaTexture, ImageSkyboxTexture, ImageTexture, Intersection, LogTexture,
                             Material, Matrix, MirrorBallSkymapTexture, MultiplyTexture, Plane,
                             SphericalCoordinatesSkymapTexture, Sphere, TransformedObject, TransformedTexture, Union,
                             union_array)

# explicit matrices (constructor order x00 x10 x20 x30 x01 x11 x21 x31 x02 x12 x22 x32)
ROT_SCALE = Matrix(0.8, -0.36, 0.48, 0.3, 0.6, 0.48, -0.64, -0.2, 0.0, 0.8, 0.6, 0.5)
SHEAR = Matrix(1.0, 0.25, 0.0, -0.1, 0.0, 1.5, 0.1, 0.05, 0.2, 0.0, 0.9, 0.0)


def zoo_images(seed=3):
    rng = np.random.default_rng(seed)
    imgs = []
    for (h, w) in [(23, 37), (16, 16), (16, 16), (16, 16), (16, 16), (16, 16), (16, 16)]:
        a = rng.uniform(0, 2, size=(h, w, 4)).astype(np.float32)
        a[..., 3] = rng.uniform(0, 1, size=(h, w)).astype(np.float32)
        imgs.append(Image(a))
    return imgs


def csg_zoo():
    diffuse = Material(ColorTexture(0.8, 0.7, 0.6), ColorTexture(1))
    glossy = Material(ColorTexture(0.9), ColorTexture(0.3))
    glass = Material(ColorTexture(0.7), ColorTexture(0), ColorTexture(0), ColorTexture(0.9, 0.95, 1.0), 1.45,
                     ColorTexture(0.8))
    mirror = Material(ColorTexture(0.99), ColorTexture(0))
    emit = Material(ColorTexture(0), ColorTexture(0), ColorTexture(1.5, 1.2, 0.9))
    sky = Material(ColorTexture(0), ColorTexture(0), ColorTexture(0.4, 0.6, 1.0))
    lens = Intersection(Sphere((0.0, 0.2, -3.2), 0.9, glass), Sphere((0.0, 0.2, -4.6), 0.9, glass))
    carved = Difference(Sphere((-1.1, -0.1, -4.0), 0.7, diffuse),
                        Union(Sphere((-0.8, 0.2, -3.4), 0.45, glossy), Plane((0, 1, 0), (0, 0.3, 0), diffuse)))
    # a hole inside, B covering A's end, B starting before A (the copyEndFromStart quirk)
    quirk = Difference(Sphere((1.2, -0.2, -4.2), 0.6, mirror), Sphere((1.0, -0.2, -3.7), 0.4, glossy))
    xf = TransformedObject(ROT_SCALE, Union(Sphere((0.4, -0.9, -4.5), 0.35, glossy),
                                            Intersection(Plane((0, -1, 0), (0, -0.7, 0), diffuse),
                                                         Sphere((0.4, -0.9, -4.5), 0.6, emit))))
    nested = TransformedObject(SHEAR, TransformedObject(ROT_SCALE, Sphere((-0.3, 1.0, -5.0), 0.4, emit)))
    floor = Plane((0, 1, 0), 1.0, diffuse)
    return union_array([lens, carved, quirk, xf, nested, floor, Plane((0, 0, 1), 50, sky)])


def texture_zoo(imgs=None):
    """Every texture class whose arithmetic is IEEE-exact (+ - * / sqrt, floor):
    bit-identical to the reference on the GPU."""
    imgs = imgs or zoo_images()
    planar = imgs[0]
    faces = imgs[1:7]
    mb = Material(ColorTexture(0), ColorTexture(0),
                  MultiplyTexture((0.5, 0.7, 0.9), MirrorBallSkymapTexture(ImageTexture(planar))))
    box = Material(ColorTexture(0), ColorTexture(0), ImageSkyboxTexture(*faces))
    alpha_sc = Material(TransformedTexture(SHEAR, ImageTexture(planar)), ImageAlphaTexture(planar))
    box_alpha = Material(ColorTexture(0.6), ImageSkyboxAlphaTexture(*faces), ImageTexture(planar))
    coord = Material(ColorTexture(0), ColorTexture(0),
                     MultiplyTexture((0.05, 0.05, 0.05),
                                     TransformedTexture(ROT_SCALE, MirrorBallSkymapTexture(CoordTexture()))))
    return union_array([
        Sphere((-0.9, 0.0, -3.5), 0.5, alpha_sc),
        Sphere((0.9, 0.0, -3.5), 0.5, box_alpha),
        Sphere((0.0, 0.8, -4.5), 0.45, coord),
        Sphere((0.0, -0.6, -3.2), 0.3, box),
        Plane((0, 0, 1), 30, mb),
        Plane((0, 1, 0), 1.2, Material(ColorTexture(0), ColorTexture(0), ImageTexture(planar))),
        Plane((0, -1, 0), 8, box),
    ])


def texture_transc_zoo(imgs=None):
    """Textures that call transcendentals (SphericalCoordinatesSkymapTexture:
    atan2f + asin; LogTexture: logf).  The GPU's libm and glibc may differ by
    an ulp, so these are held to a tolerance, not bits."""
    imgs = imgs or zoo_images()
    planar = imgs[0]
    sph = Material(ColorTexture(0), ColorTexture(0), SphericalCoordinatesSkymapTexture(ImageTexture(planar)))
    logm = Material(ColorTexture(0.6), ColorTexture(0.8), LogTexture(ImageTexture(planar)))
    coord = Material(ColorTexture(0), ColorTexture(0),
                     MultiplyTexture((0.05, 0.05, 0.05),
                                     TransformedTexture(ROT_SCALE, SphericalCoordinatesSkymapTexture(CoordTexture()))))
    return union_array([
        Sphere((-0.6, 0.0, -3.5), 0.5, logm),
        Sphere((0.6, 0.5, -4.5), 0.45, coord),
        Plane((0, 1, 0), 1.2, sph),
        Plane((0, 0, 1), 30, sph),
    ])


def random_rays(n, seed=9, spread=1.0):
    rng = np.random.default_rng(seed)
    o = rng.uniform(-spread, spread, size=(n, 3)).astype(np.float32) * np.float32(0.5)
    o[:, 2] += np.float32(-1.0)
    d = rng.normal(size=(n, 3)).astype(np.float32)
    d[:, 2] = -np.abs(d[:, 2]) - np.float32(0.2)
    d *= rng.uniform(0.5, 3000, size=(n, 1)).astype(np.float32)
    return np.concatenate([o, d], axis=1).astype(np.float32)


def trace_rays_input(n, seed=17):
    """Caller rays for traceRay (n x 7: origin, direction, strength): random
    rays near the scenes (random_rays), a quarter of them camera-like from the
    origin, strengths from below eps (traceRay returns the emission alone,
    include/path-trace.h:105-108) up to 3 (more scatter children)."""
    rng = np.random.default_rng(seed)
    r = random_rays(n, seed=seed)
    r[: n // 4, :3] = 0.0
    # mostly short directions: eps = 1e-3 applies to t, so |d| ~ 3000 skips all
    # the scene within 3 units of the origin
    d = r[:, 3:6] / np.linalg.norm(r[:, 3:6], axis=1, keepdims=True)
    # half of them aimed into the box around the demo spheres (z -4.6 .. -3.2)
    tgt = rng.uniform([-1.6, -0.7, -4.6], [1.6, 0.7, -3.2], size=(n, 3)).astype(np.float32)
    aim = rng.random(n) < 0.5
    v = tgt - r[:, :3]
    d[aim] = (v / np.linalg.norm(v, axis=1, keepdims=True))[aim]
    r[:, 3:6] = d * rng.choice([0.7, 1.0, 4.0, 30.0, 2000.0], size=(n, 1), p=[.25, .35, .2, .15, .05])
    s = rng.uniform(0.0, 3.0, size=(n, 1)).astype(np.float32)
    s[rng.random(n) < 0.15] = np.float32(0.0005)
    s[rng.random(n) < 0.25] = np.float32(1.0)
    return np.concatenate([r, s], axis=1).astype(np.float32)


# (name, builder, W, H, spp, depth) of the per-sample render goldens
RENDER_CASES = [
    ("p0", "scene_p0", 32, 24, 3, 4),
    ("p1", "scene_p1", 32, 24, 3, 8),
    ("csg", "csg_zoo", 32, 24, 3, 6),
    ("tex", "texture_zoo", 32, 24, 3, 5),
    ("texm", "texture_transc_zoo", 32, 24, 3, 5),
]
# every case bit for bit: the spherical map's atan2f / asinf and LogTexture's
# logf are glibc's algorithms restated on the device (tests/test_libm.py)
EXACT_CASES = list(RENDER_CASES)
# (builder, depth) of scenes only the GPU tests render (against the oracle, no goldens)
GPU_ONLY_CASES = [("union_zoo", 6)]


def build(name):
    from pathtrace import scenes
    if hasattr(scenes, name):
        return getattr(scenes, name)()
    return globals()[name]()


def occlude_box(variant="box"):
    """Union-only scene for the plane-occluder dark test (tests/test_occlude.py):
    diffuse, glossy and mirror spheres over a ground plane inside a box of
    emissive half-spaces 3 from the origin on x and y and 8 on z, so ground
    entries fall on both sides of the emitters' bound; "emissive_sphere" adds a
    lit sphere (no bound, no claim), "tilted" tilts the ground (not
    axis-aligned, no claim)."""
    diffuse = Material(ColorTexture(0.8), ColorTexture(1))
    glossy = Material(ColorTexture(0.7), ColorTexture(0.5))
    mirror = Material(ColorTexture(0.99), ColorTexture(0))
    sky = Material(ColorTexture(0), ColorTexture(0), ColorTexture((0.5, 0.7, 1.0)))
    ground = Plane((0.05, 1, 0), 0.7, diffuse) if variant == "tilted" else Plane((0, 1, 0), 0.7, diffuse)
    objs = [Sphere((-0.8, -0.2, -4), 0.5, diffuse), Sphere((0.8, -0.25, -4), 0.45, glossy),
            Sphere((0, 0.1, -5), 0.5, mirror), ground]
    if variant == "emissive_sphere":
        objs.append(Sphere((0, 1.5, -4.5), 0.3, Material(ColorTexture(0), ColorTexture(0), ColorTexture(3.0))))
    for n in [(0, 0, -1), (0, 0, 1), (0, -1, 0), (0, 1, 0), (1, 0, 0), (-1, 0, 0)]:
        objs.append(Plane(n, 8 if n[2] else 3, sky))
    return union_array(objs)


def union_zoo():
    """Union-only scene for the union rule (pt_device.h union_min_ok): an
    emissive box of six inward half-spaces, spheres that overlap, nest and
    coincide exactly (equal spans: ties the rule must hand to the pairwise
    checks), a ground plane with an exact duplicate, and an emissive sphere
    inside a glass one."""
    diffuse = Material(ColorTexture(0.8, 0.7, 0.6), ColorTexture(1))
    glossy = Material(ColorTexture(0.9), ColorTexture(0.3))
    glass = Material(ColorTexture(0.7), ColorTexture(0), ColorTexture(0), ColorTexture(0.9, 0.95, 1.0), 1.45,
                     ColorTexture(0.8))
    mirror = Material(ColorTexture(0.99), ColorTexture(0))
    emit = Material(ColorTexture(0), ColorTexture(0), ColorTexture(1.5, 1.2, 0.9))
    sky = Material(ColorTexture(0), ColorTexture(0), ColorTexture(0.4, 0.6, 1.0))
    objs = [Sphere((-1.0, 0.0, -4.0), 0.6, diffuse), Sphere((-0.4, 0.1, -4.1), 0.6, glossy),  # overlapping
            Sphere((1.0, 0.0, -4.0), 0.6, mirror), Sphere((1.0, 0.0, -4.0), 0.6, diffuse),     # coincident
            Sphere((0.0, 0.9, -4.5), 0.7, glass), Sphere((0.0, 0.9, -4.5), 0.25, emit),       # nested
            Plane((0, 1, 0), 0.7, diffuse), Plane((0, 1, 0), 0.7, glossy)]                    # duplicate ground
    for n in [(0, 0, -1), (0, 0, 1), (0, -1, 0), (0, 1, 0), (1, 0, 0), (-1, 0, 0)]:
        objs.append(Plane(n, 60, sky))
    return union_array(objs)


def scatter_zoo():
    """Scatter loops a lane walks whole (pt_scene_set_lane_scatter): small
    glossy loops (N = 10^4 strength sc <= 64 children, which recurse), a bright
    diffuse sphere whose children recurse in part (matBrightDiffuseWhite's
    reflectance 8), a dim diffuse floor (a plain burst: the wave's), glass and a
    mirror, under a sky whose upper wall emits nothing (zero terms among the
    non-zero ones)."""
    tiny = Material(ColorTexture(0.9, 0.8, 0.7), ColorTexture(0.0064))
    small = Material(ColorTexture(0.6), ColorTexture(0.002))
    bright = Material(ColorTexture(8), ColorTexture(1))
    dim = Material(ColorTexture(0.3, 0.25, 0.2), ColorTexture(1))
    glass = Material(ColorTexture(0.7), ColorTexture(0), ColorTexture(0), ColorTexture(0.9, 0.95, 1.0), 1.45,
                     ColorTexture(0.8))
    mirror = Material(ColorTexture(0.99), ColorTexture(0))
    emit = Material(ColorTexture(0), ColorTexture(0), ColorTexture(1.5, 1.2, 0.9))
    sky = Material(ColorTexture(0), ColorTexture(0), ColorTexture(0.4, 0.6, 1.0))
    black = Material(ColorTexture(0), ColorTexture(0), ColorTexture(0))
    return union_array([
        Sphere((-1.0, 0.0, -4.0), 0.6, tiny), Sphere((0.3, -0.3, -3.6), 0.35, bright),
        Sphere((1.1, 0.1, -4.2), 0.55, small), Sphere((-0.2, 0.7, -4.8), 0.5, glass),
        Sphere((0.9, 0.9, -5.0), 0.4, mirror), Sphere((-1.2, 1.0, -5.5), 0.3, emit),
        Plane((0, 1, 0), 0.7, dim), Plane((0, -1, 0), 3.0, black), Plane((0, 0, 1), 30, sky)])


def texture_points(n=2048, seed=13):
    """Lookup points for the texture query goldens (pt_tex_eval): random points
    in a box, unit directions (the sky maps' domain), points on the cube-face
    diagonals and axes (skybox face ties), exact zeros and far points."""
    rng = np.random.default_rng(seed)
    box = rng.uniform(-3, 3, size=(n // 2, 3))
    d = rng.normal(size=(n // 4, 3))
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    ties = rng.choice([-1.0, 1.0], size=(n // 8, 3)) * rng.uniform(0.1, 2, size=(n // 8, 1))
    ties[: n // 16, rng.integers(0, 3)] = 0.0
    axes = np.concatenate([np.eye(3), -np.eye(3), np.zeros((1, 3))]) * np.array([[1.0], [2.5], [0.3], [1.0], [7.0],
                                                                                [0.5], [1.0]])
    far = rng.normal(size=(n - len(box) - len(d) - len(ties) - len(axes), 3)) * 1e4
    return np.concatenate([box, d, ties, axes, far]).astype(np.float32)


# scenes of the texture query goldens (tests/golden/tex_eval.npz)
TEX_EVAL_SCENES = ["texture_zoo", "texture_transc_zoo"]
