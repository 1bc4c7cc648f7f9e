"""The benchmark / parity scenes, built through the
reference-mirroring scene API.

Materials are the demo's (reference src/test.cpp:109-118):
  diffuse  Material(ColorTexture(0.8), ColorTexture(1))
  mirror   Material(ColorTexture(0.99), ColorTexture(0))
  glass    Material(ColorTexture(0.7), ColorTexture(0), ColorTexture(0), ColorTexture(0.9), 1.3, ColorTexture(1))
  emitW    Material(ColorTexture(0), ColorTexture(0), ColorTexture(2))
  sky      Material(ColorTexture(0), ColorTexture(0), ColorTexture(0.5, 0.7, 1.0))
Camera convention of the reference caller (src/test.cpp:450): screen_w = W,
screen_h = H, screen_dist = 2 * min(W, H), origin 0, looking down -z.
"""
from __future__ import annotations

import math
import os
from dataclasses import dataclass, field
from typing import Callable, Dict

import numpy as np

from .scene import (ColorTexture, Difference, Image, ImageSkyboxTexture, ImageTexture, Intersection, Material,
                    Matrix, MirrorBallSkymapTexture, MultiplyTexture, Plane, SphericalCoordinatesSkymapTexture,
                    Sphere, TransformedTexture, Union, transform_material, union_array)


def materials():
    return {
        "diffuse": Material(ColorTexture(0.8), ColorTexture(1)),
        "mirror": Material(ColorTexture(0.99), ColorTexture(0)),
        "glass": Material(ColorTexture(0.7), ColorTexture(0), ColorTexture(0), ColorTexture(0.9), 1.3,
                          ColorTexture(1)),
        "emitW": Material(ColorTexture(0), ColorTexture(0), ColorTexture(2)),
        "sky": Material(ColorTexture(0), ColorTexture(0), ColorTexture(0.5, 0.7, 1.0)),
        "diamond": Material(ColorTexture(0.2), ColorTexture(0), ColorTexture(0), ColorTexture(0.9), 2.419,
                            ColorTexture(1)),
        "brightDiffuse": Material(ColorTexture(8), ColorTexture(1)),
    }


def scene_p0():
    """C1 / P0: three spheres (diffuse, mirror, glass) over an emissive floor."""
    m = materials()
    return Union(Union(Sphere((-1, 0, -4), .5, m["diffuse"]), Sphere((1, 0, -4), .5, m["mirror"])),
                 Union(Sphere((0, .3, -5), .5, m["glass"]), Plane((0, 1, 0), .5, m["emitW"])))


def scene_p1():
    """C3 / P1 (north star): union/difference CSG of six spheres + constant sky wall.
    Exercises the Difference quirk of reference src/difference.cpp:124-130."""
    m = materials()
    left = Difference(Union(Sphere((-1, 0, -4), .6, m["diffuse"]), Sphere((-.5, 0, -4), .6, m["diffuse"])),
                      Sphere((-.7, .3, -3.6), .4, m["diffuse"]))
    right = Difference(Union(Sphere((1, 0, -4), .6, m["glass"]), Sphere((1.4, .2, -4.2), .5, m["mirror"])),
                       Sphere((1, 0, -3.4), .3, m["glass"]))
    return Union(left, Union(right, Plane((0, 0, 1), 200, m["sky"])))


# The reference's own input images, shipped as data:
# test2.hdr (640x480) stands in for the missing stpeters_probe.hdr (C2),
# test.hdr (1280x1509) for the missing Serpentine_Valley_3k.hdr (C5), and
# sky01/*.png (6 x 877^2) is the skybox of makeSkyBox (src/test.cpp:88-95).
ASSETS = os.path.join(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))), "assets")
_images: Dict[str, Image] = {}


def asset_image(name: str) -> Image:
    """Image(fileName) of a reference asset, loaded once per process by the
    product's own loaders (pt_image_load_hdr / pt_image_load_png)."""
    if name not in _images:
        _images[name] = Image(path=os.path.join(ASSETS, name))
    return _images[name]


def procedural_env(w: int, h: int, seed: int = 7) -> Image:
    """Deterministic synthetic HDR environment map (substitute for the missing
    stpeters_probe.hdr / Serpentine_Valley_3k.hdr): a sky
    gradient with a few bright 'sun' blobs and a checker, RGBA32F."""
    ys, xs = np.mgrid[0:h, 0:w].astype(np.float32)
    u = xs / np.float32(w)
    v = ys / np.float32(h)
    r = 0.3 + 0.7 * (1 - v)
    g = 0.4 + 0.5 * (1 - v) ** 2
    b = 0.6 + 0.4 * np.sqrt(1 - v)
    checker = ((xs // 16 + ys // 16) % 2).astype(np.float32) * 0.15
    rng = np.random.default_rng(seed)
    sun = np.zeros_like(u)
    for _ in range(4):
        cx, cy, rad, amp = rng.uniform(0, 1), rng.uniform(0, 0.5), rng.uniform(0.02, 0.06), rng.uniform(5, 40)
        sun += amp * np.exp(-((u - cx) ** 2 + (v - cy) ** 2) / (rad * rad))
    img = np.stack([r + checker + sun, g + checker + 0.8 * sun, b + checker + 0.6 * sun, np.ones_like(u)], -1)
    return Image(img.astype(np.float32))


def procedural_face(size: int, face: int) -> Image:
    ys, xs = np.mgrid[0:size, 0:size].astype(np.float32)
    base = np.float32(0.15 + 0.12 * face)
    stripes = ((xs // (8 + face) + ys // 8) % 2).astype(np.float32) * 0.3
    r = base + stripes
    g = base * 0.8 + stripes * (face % 3) * 0.4
    b = base * 1.2 + (ys / size) * 0.5
    img = np.stack([r, g, b, np.ones_like(r)], -1).astype(np.float32)
    return Image(img)


def scene_c2(procedural: bool = False, full_mix: bool = True):
    """C2: eight spheres of the demo material mix over a ground plane inside six
    inward sky half-spaces at distance 200 carrying a mirror-ball sky map
    (reference makeSkyMirrorSphere, src/test.cpp:97-100 and :134-140) of
    test2.hdr (procedural=True: a synthetic 640x480 map, for CPU-only tests).
    The mix (src/test.cpp:109-118) includes matBrightDiffuseWhite (reflectance
    8, |rc| = 13.9) on the fourth sphere: the children of a diffuse bounce off
    it have strength up to 13.9e-4 > eps, so about a quarter of its 10^4
    children recurse (full_mix=False swaps in plain diffuse, the round-2 C2)."""
    m = materials()
    env = procedural_env(640, 480) if procedural else asset_image("test2.hdr")
    sky = Material(ColorTexture(0), ColorTexture(0),
                   MultiplyTexture((1, 1, 1), MirrorBallSkymapTexture(ImageTexture(env))))
    mats = [m["diffuse"], m["mirror"], m["glass"], m["brightDiffuse"] if full_mix else m["diffuse"], m["diamond"],
            m["mirror"], m["glass"], m["diffuse"]]
    objs = []
    for k in range(8):
        ang = 2 * math.pi * k / 8
        objs.append(Sphere((1.6 * math.cos(ang), -0.2 + 0.1 * (k % 3), -5 + 1.6 * math.sin(ang)), 0.45, mats[k]))
    objs.append(Plane((0, 1, 0), 0.7, m["diffuse"]))
    for n in [(0, 0, -1), (0, 0, 1), (0, -1, 0), (0, 1, 0), (1, 0, 0), (-1, 0, 0)]:
        objs.append(Plane(n, 200, sky))
    return union_array(objs)


def scene_c5(procedural: bool = False):
    """C5: the reference demo world (src/test.cpp:107-145) with test.hdr in
    place of Serpentine_Valley_3k.hdr (kept under rotateX(pi/2) and scale 0.01)
    plus a sphere whose emissive is an ImageSkyboxTexture of sky01/*.png
    (makeSkyBox, src/test.cpp:88-95).  procedural=True swaps in small
    synthetic images (CPU-only tests)."""
    m = materials()
    env = procedural_env(1024, 512, seed=11) if procedural else asset_image("test.hdr")
    sky_sph = Material(ColorTexture(0), ColorTexture(0),
                       MultiplyTexture((0.01, 0.01, 0.01), SphericalCoordinatesSkymapTexture(ImageTexture(env))))
    sky = transform_material(Matrix.rotateX(2 * math.pi / 4), sky_sph)
    diffuse, glass, emitW = m["diffuse"], m["glass"], m["emitW"]
    dw = transform_material(Matrix.translate(-1, 0, 4), diffuse)
    ew = transform_material(Matrix.translate(-1, 0, 4), emitW)
    if procedural:
        faces = [procedural_face(128, k) for k in range(6)]
    else:
        faces = [asset_image("sky01/%s.png" % f) for f in ("top", "bottom", "left", "right", "front", "back")]
    skybox = Material(ColorTexture(0), ColorTexture(0), ImageSkyboxTexture(*faces))

    def make_lens(position, orientation, radius, sphere_radius, material):
        dist = math.sqrt(sphere_radius * sphere_radius - radius * radius)
        o = np.array(orientation, dtype=np.float32)
        o = o / np.float32(np.sqrt(np.float32((o[0] * o[0] + o[1] * o[1]) + o[2] * o[2])))
        p = np.array(position, dtype=np.float32)
        return Intersection(Sphere(p + o * np.float32(dist), sphere_radius, material),
                            Sphere(p - o * np.float32(dist), sphere_radius, material))

    objs = [
        Sphere((1, 0, -4), 0.2, dw),
        Intersection(Sphere((1, 0, -4), 0.2 * 5, glass),
                     Union(Plane((-1, 0, -0.7), (1, 0, -4), glass), Sphere((1, 0, -4), 0.2, ew))),
        Sphere((-1, 0, -4), 0.2, diffuse),
        Plane((0, 0, -1), 200, sky),
        Plane((0, 0, 1), 200, sky),
        Plane((0, -1, 0), 200, sky),
        Plane((0, 1, 0), 200, sky),
        Plane((1, 0, 0), 200, sky),
        Plane((-1, 0, 0), 200, sky),
        make_lens((-2.5 / 4, 0, -2.5), (-1, 0, -4), 0.5, 1, glass),
        Sphere((0, 1.2, -6), 0.7, skybox),
    ]
    return union_array(objs)


@dataclass
class Config:
    name: str
    width: int
    height: int
    spp: int
    depth: int
    scene: Callable
    gpus: int = 1
    note: str = ""
    wg_per_cu: int = 0  # pt_scene_set_occupancy (0 = as many as LDS allows)
    fast_spine: bool = False  # pt_scene_set_fast_spine
    lane_walk: int = 0  # pt_scene_set_lane_walk (register frames; 0 = off)
    lane_scatter: bool = False  # pt_scene_set_lane_scatter

    def device_scene(self, procedural: bool = False, root=None):
        """The config's scene (or `root`) as a DeviceScene with the config's
        occupancy and walk settings."""
        from . import DeviceScene
        if root is None:
            root = self.scene(procedural=True) if procedural else self.scene()
        return DeviceScene(root, workgroups_per_cu=self.wg_per_cu, fast_spine=self.fast_spine,
                           lane_walk=self.lane_walk, lane_scatter=self.lane_scatter)

    @property
    def screen(self):
        return (float(self.width), float(self.height), float(2 * min(self.width, self.height)))


CONFIGS: Dict[str, Config] = {
    "C1": Config("C1", 256, 256, 16, 4, scene_p0, note="plumbing; CPU reference path"),
    # C2 without matBrightDiffuseWhite: with it the reference's own cost per
    # sample has no practical bound (C2_FULL below)
    # C2 with span-first spine queries since round 4 (same box, 65 536 hashed
    # pixels at 16 spp: 4.83 -> 4.91 Msamples/s)
    "C2": Config("C2", 1280, 720, 256, 16, lambda procedural=False: scene_c2(procedural, full_mix=False),
                 note="8 spheres (no matBrightDiffuseWhite) + plane + mirror-ball env (test2.hdr)", fast_spine=True),
    # C3/C4: span-first spine queries (same-box A/B at 1024 spp: 156.3 -> 157.2
    # Msamples/s; round 2's kernel lost 0.9 % with them)
    "C3": Config("C3", 1920, 1080, 1024, 8, scene_p1, note="north star: 6-sphere union/difference CSG",
                 fast_spine=True),
    "C4": Config("C4", 1920, 1080, 4096, 8, scene_p1, gpus=8, note="C3 scene over 8 GPUs + RCCL framebuffer reduce",
                 fast_spine=True),
    # C5 at 2 workgroups per CU: its 14-primitive tree spills 1032 VGPRs at the
    # default cap of 128 (119 -> 277 Msamples/s on one MI355X, round 2).  Its
    # glass-ball trees have no scatter loop: lanes walk them with register
    # frames instead of the wave (bench-like subset at 256 spp 685 -> 2330
    # Msamples/s, glass disk 65 -> 708; 3 frames 2311, 4 frames 2164).  Since
    # the zero-weight skip (round 6) a sky hit needs no frame for its mirror
    # child, and one frame is best: 19.09 -> 19.36 G on the bench subset
    # (2 frames; 3: 18.53; profiles/round6/ab_lane_walk_c5_r6.txt)
    "C5": Config("C5", 3840, 2160, 8192, 16, scene_c5, gpus=8,
                 note="demo world + test.hdr spherical env + sky01 skybox", wg_per_cu=2, fast_spine=True,
                 lane_walk=1),
}


def scene_c2_plain(procedural: bool = False):
    """C2 without matBrightDiffuseWhite (plain diffuse on the fourth sphere):
    the benchmarked C2, the scene of tests/golden/config_C2.npz."""
    return scene_c2(procedural, full_mix=False)


C2_PLAIN = CONFIGS["C2"]

# C2 with the reference's full material mix (src/test.cpp:109-118): supported
# bit for bit (lanes walk the bright sphere's chains of small recursing loops,
# pt_scene_set_lane_scatter) and tested on pixel subsets, but not a frame
# workload: behind the glass sphere's silhouette a single sample's ray tree
# grows ~3.6x per depth level -- pixel (544, 360) costs 3.03e6 queries at
# depth 8 and 1.17e7 at depth 9 in the UNMODIFIED reference (oracle/_ref/ptref,
# 6.1 s on one core), ~9e10 extrapolated to depth 16 (~14 h on one core for
# one sample, sequential in its engine's draws)
C2_FULL = Config("C2full", 1280, 720, 256, 16, scene_c2,
                 note="8 spheres (full demo mix) + plane + mirror-ball env (test2.hdr)", lane_scatter=True)
