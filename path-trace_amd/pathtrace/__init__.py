"""pathtrace -- MI355X-native renderer for the reference's per-pixel
Monte-Carlo path (tracePixel -> traceRay -> CSG span queries -> shading).

Python mirror of the reference's scene API (pathtrace.scene) on top of the
C-ABI library libpt.so (include/pt/pt.h), whose megakernel runs on gfx950.

    from pathtrace import *
    world = Union(Sphere((0, 0, -4), .5, Material(ColorTexture(.8), ColorTexture(1))),
                  Plane((0, 1, 0), .5, Material(ColorTexture(0), ColorTexture(0), ColorTexture(2))))
    img = render(world, 256, 256, spp=16, depth=4)        # H x W x 3 float32 (tracePixel means)
    write_hdr("out.hdr", img); write_bmp("out.bmp", img)
"""
from __future__ import annotations

import ctypes
from typing import Optional, Sequence

import numpy as np

from . import _lib
from ._lib import PT_ORDER_FAST, PT_ORDER_REFERENCE, PtError, RenderParams, RenderStats, TraceParams, load_hdr, \
    load_png, write_bmp, write_hdr
from .scene import (ColorTexture, CoordTexture, DeviceObject, DeviceTexture, Difference, Image, ImageAlphaTexture, ImageSkyboxAlphaTexture,
                    ImageSkyboxTexture, ImageTexture, Intersection, LogTexture, Material, Matrix,
                    MirrorBallSkymapTexture, MultiplyTexture, Object, Plane, SphericalCoordinatesSkymapTexture,
                    Sphere, Texture, TransformedObject, TransformedTexture, Union, invert, to_text,
                    transform_material, transform_object, transform_texture, union_array)

__all__ = [n for n in dir() if not n.startswith("_")] + ["DeviceScene", "render", "render_device", "prepare",
                                                         "trace_rays"]

ORDERS = {"fast": PT_ORDER_FAST, "reference": PT_ORDER_REFERENCE,
          "strict": PT_ORDER_REFERENCE,
          "group64": PT_ORDER_FAST}  # deprecated name of "fast" (rounds 1-2)


class DeviceScene:
    """A pt_scene built from a Python scene graph through the C-ABI
    constructors (one pt_* call per reference constructor)."""

    def __init__(self, root: Object, workgroups_per_cu: int = 0, fast_spine: bool = False, lane_walk: int = 0,
                 lane_scatter: bool = False, split: bool = True):
        L = _lib.lib()
        self._h = L.pt_scene_create()
        if not self._h:
            raise PtError("pt_scene_create failed")
        if workgroups_per_cu:
            _lib.check(L.pt_scene_set_occupancy(self._h, int(workgroups_per_cu)))
        if fast_spine:
            _lib.check(L.pt_scene_set_fast_spine(self._h, 1))
        if lane_walk:
            _lib.check(L.pt_scene_set_lane_walk(self._h, int(lane_walk)))
        if lane_scatter:
            _lib.check(L.pt_scene_set_lane_scatter(self._h, 1))
        if not split:
            _lib.check(L.pt_scene_set_split(self._h, 0))
        self._img = {}
        self._mat = {}
        self.root = root
        _lib.check(L.pt_set_root(self._h, self._obj(root)))

    @classmethod
    def from_text(cls, text: str) -> "DeviceScene":
        """A pt_scene loaded from the plain-text scene format (pt_scene_from_text);
        its textures / materials / objects get ids in file order."""
        self = cls.__new__(cls)
        L = _lib.lib()
        self._h = L.pt_scene_create()
        if not self._h:
            raise PtError("pt_scene_create failed")
        self._img, self._mat, self.root = {}, {}, None
        _lib.check(L.pt_scene_from_text(self._h, text.encode()))
        return self

    def __del__(self):
        h = getattr(self, "_h", None)
        if h:
            _lib.lib().pt_scene_destroy(h)
            self._h = None

    @property
    def handle(self):
        return self._h

    def _image(self, im: Image) -> int:
        k = id(im)
        if k not in self._img:
            d = np.ascontiguousarray(im.data, dtype=np.float32)
            self._img[k] = _lib.check(_lib.lib().pt_image_from_rgba32f(self._h, d.ctypes.data, d.shape[1],
                                                                       d.shape[0]))
        return self._img[k]

    def _tex(self, t: Texture) -> int:
        L, h, c = _lib.lib(), self._h, _lib.check
        if isinstance(t, ColorTexture):
            return c(L.pt_tex_color(h, *[float(v) for v in t.color]))
        if isinstance(t, CoordTexture):
            return c(L.pt_tex_coord(h))
        if isinstance(t, DeviceTexture):
            prm = (ctypes.c_float * max(1, len(t.params)))(*t.params)
            return c(L.pt_tex_device(h, t.color_body.encode(), t.value_body.encode() if t.value_body else None,
                                     prm, len(t.params)))
        if isinstance(t, ImageSkyboxAlphaTexture):
            return c(L.pt_tex_skybox_alpha(h, *[self._image(f) for f in t.faces]))
        if isinstance(t, ImageSkyboxTexture):
            return c(L.pt_tex_skybox(h, *[self._image(f) for f in t.faces]))
        if isinstance(t, ImageAlphaTexture):
            return c(L.pt_tex_image_alpha(h, self._image(t.image)))
        if isinstance(t, ImageTexture):
            return c(L.pt_tex_image(h, self._image(t.image)))
        if isinstance(t, MultiplyTexture):
            inner = self._tex(t.t)
            return c(L.pt_tex_multiply(h, *[float(v) for v in t.factor], inner))
        if isinstance(t, TransformedTexture):
            inner = self._tex(t.t)
            return c(L.pt_tex_transformed(h, _lib._f12(t.matrix.m), inner))
        if isinstance(t, MirrorBallSkymapTexture):
            return c(L.pt_tex_mirrorball(h, self._tex(t.t)))
        if isinstance(t, SphericalCoordinatesSkymapTexture):
            return c(L.pt_tex_spherical(h, self._tex(t.t)))
        if isinstance(t, LogTexture):
            return c(L.pt_tex_log(h, self._tex(t.t)))
        raise TypeError("unsupported texture %r" % (t,))

    def _material(self, m: Material) -> int:
        k = id(m)
        if k not in self._mat:
            ids = [self._tex(t) for t in m.textures()]
            self._mat[k] = _lib.check(_lib.lib().pt_material(self._h, ids[0], ids[1], ids[2], ids[3],
                                                              float(m.ior), ids[4]))
        return self._mat[k]

    def _obj(self, o: Object) -> int:
        L, h, c = _lib.lib(), self._h, _lib.check
        if isinstance(o, Sphere):
            return c(L.pt_sphere(h, *[float(v) for v in o.center], float(o.r), self._material(o.material)))
        if isinstance(o, Plane):
            return c(L.pt_plane(h, *[float(v) for v in o.normal], float(o.d), self._material(o.material)))
        if isinstance(o, DeviceObject):
            prm = (ctypes.c_float * max(1, len(o.params)))(*o.params)
            return c(L.pt_object_device(h, o.span_body.encode(), o.normal_body.encode(), prm, len(o.params),
                                        self._material(o.material)))
        if isinstance(o, (Union, Intersection, Difference)):
            op = {Union: 0, Intersection: 1, Difference: 2}[type(o)]
            a = self._obj(o.a)
            b = self._obj(o.b)
            return c(L.pt_csg(h, op, a, b))
        if isinstance(o, TransformedObject):
            ch = self._obj(o.o)
            return c(L.pt_transformed(h, _lib._f12(o.matrix.m), ch))
        raise TypeError("unsupported object %r" % (o,))

    def query_spans(self, rays, max_spans: int = 16, device: int = 0):
        """obj->makeSpanIterator() over the root for each ray (n x 6: origin,
        direction), evaluated on the device (pt_query_spans): returns
        (counts[n], spans[n, max_spans, 10] as float32 words: t, normal,
        material id (int32 bits) for the start, then for the end)."""
        rays = np.ascontiguousarray(rays, dtype=np.float32).reshape(-1, 6)
        n = len(rays)
        out = np.zeros((n, max_spans, 10), dtype=np.float32)
        counts = np.zeros(n, dtype=np.int32)
        _lib.check(_lib.lib().pt_query_spans(self._h, -1, rays.ctypes.data, n, int(max_spans), out.ctypes.data,
                                             counts.ctypes.data, int(device)))
        return counts, out

    def tex_eval(self, texture, points, device: int = 0):
        """Texture::getColor / getFloat at n points (n x 3) on the device
        (pt_tex_eval) of a Texture (flattened into this scene) or a texture id:
        returns (rgb[n, 3], value[n])."""
        pts = np.ascontiguousarray(points, dtype=np.float32).reshape(-1, 3)
        rgb = np.zeros((len(pts), 3), dtype=np.float32)
        val = np.zeros(len(pts), dtype=np.float32)
        tid = int(texture) if isinstance(texture, (int, np.integer)) else self._tex(texture)
        _lib.check(_lib.lib().pt_tex_eval(self._h, tid, pts.ctypes.data, len(pts), rgb.ctypes.data,
                                          val.ctypes.data, int(device)))
        return rgb, val

    def compile_queries(self, textures=()) -> None:
        """Compile the query modules -- the root's span query and each texture's
        (Texture objects or ids) -- without a device."""
        _lib.check(_lib.lib().pt_query_compile(self._h, -1, -1))
        for t in textures:
            tid = int(t) if isinstance(t, (int, np.integer)) else self._tex(t)
            _lib.check(_lib.lib().pt_query_compile(self._h, -2, tid))

    def kernel_key(self, depth: int) -> str:
        """The code-object key of this scene's render kernel at `depth`
        (pt_scene_kernel_key: source + compiler options + hiprtc version)."""
        k = _lib.lib().pt_scene_kernel_key(self._h, depth).decode()
        if not k:
            raise PtError(_lib.lib().pt_last_error().decode())
        return k

    def compile_rays(self, depth: int) -> None:
        """Compile pt_trace_rays' module for this scene and depth (no device)."""
        _lib.check(_lib.lib().pt_trace_compile(self._h, depth))

    def compile(self, depth: int) -> str:
        _lib.check(_lib.lib().pt_scene_compile(self._h, depth))
        return _lib.lib().pt_scene_kernel_key(self._h, depth).decode()


def make_params(width, height, spp, depth, screen=None, seed=0x5EED, order="fast", device=0, pixels=None,
                max_buffer_bytes=0, grid_width=0, sample_begin=0, sum_only=False):
    sw, sh, dist = screen if screen is not None else (float(width), float(height), float(2 * min(width, height)))
    p = RenderParams()
    p.width, p.height, p.spp, p.depth = int(width), int(height), int(spp), int(depth)
    p.screen_w, p.screen_h, p.screen_dist = float(sw), float(sh), float(dist)
    p.seed = int(seed)
    p.order = ORDERS[order] if isinstance(order, str) else int(order)
    p.device = int(device)
    keep = None
    if pixels is not None:
        keep = np.ascontiguousarray(np.asarray(pixels, dtype=np.int32))
        p.pixels = keep.ctypes.data_as(ctypes.POINTER(ctypes.c_int32))
        p.npixels = len(keep)
    else:
        p.pixels = None
        p.npixels = 0
    p.max_buffer_bytes = int(max_buffer_bytes)
    p.grid_width = int(grid_width)
    p.sample_begin = int(sample_begin)
    p.sum_only = 1 if sum_only else 0
    return p, keep


def render(scene, width: int, height: int, spp: int, depth: int, screen=None, seed: int = 0x5EED,
           order="fast", pixels: Optional[Sequence[int]] = None, device: int = 0, stats: bool = False,
           max_buffer_bytes: int = 0, sample_begin: int = 0, sum_only: bool = False):
    """tracePixel means for every pixel (H x W x 3), or for `pixels` (n x 3);
    with sum_only, the per-pixel sums of samples sample_begin .. + spp - 1."""
    ds = scene if isinstance(scene, DeviceScene) else DeviceScene(scene)
    p, keep = make_params(width, height, spp, depth, screen, seed, order, device, pixels, max_buffer_bytes,
                          sample_begin=sample_begin, sum_only=sum_only)
    n = (len(keep) if keep is not None else width * height)
    out = np.zeros((n, 3), dtype=np.float32)
    st = RenderStats()
    _lib.check(_lib.lib().pt_render(ds.handle, ctypes.byref(p), out.ctypes.data, ctypes.byref(st)))
    if keep is None:
        out = out.reshape(height, width, 3)
    return (out, st.as_dict()) if stats else out


def trace_rays(scene, rays, depth: int, spp: int = 1, seed: int = 0x5EED, order="fast", device: int = 0,
               sample_begin: int = 0, ray_begin: int = 0, stats: bool = False):
    """traceRay(ray, it, depth, engine, strength) (include/path-trace.h:58-165)
    for each row of rays (n x 7 float32: origin, direction, strength; n x 6
    takes strength 1), on the device in one launch (pt_trace_rays): the mean of
    spp samples per ray, sample s of ray k drawing from the engine keyed
    (seed, ray_begin + k, sample_begin + s).  Returns n x 3 float32."""
    ds = scene if isinstance(scene, DeviceScene) else DeviceScene(scene)
    r = np.asarray(rays, dtype=np.float32)
    if r.ndim == 2 and r.shape[1] == 6:
        r = np.concatenate([r, np.ones((len(r), 1), dtype=np.float32)], axis=1)
    r = np.ascontiguousarray(r.reshape(-1, 7))
    tp = TraceParams()
    tp.spp, tp.depth, tp.seed = int(spp), int(depth), int(seed)
    tp.order = ORDERS[order] if isinstance(order, str) else int(order)
    tp.device, tp.sample_begin, tp.max_buffer_bytes, tp.ray_begin = int(device), int(sample_begin), 0, int(ray_begin)
    out = np.zeros((len(r), 3), dtype=np.float32)
    st = RenderStats()
    _lib.check(_lib.lib().pt_trace_rays(ds.handle, ctypes.byref(tp), r.ctypes.data, len(r), out.ctypes.data,
                                        ctypes.byref(st)))
    return (out, st.as_dict()) if stats else out


def render_adaptive(scene, width: int, height: int, spp: int, depth: int, screen=None, seed: int = 0x5EED,
                    order="fast", block_size: int = 0, max_interp: int = 0, min_delta: float = 0.0, device: int = 0,
                    exact_batches: bool = False):
    """The reference demo's adaptive image formation (RenderBlock::renderSquare,
    src/test.cpp:423-507) on the GPU: returns (H x W x 3 image, info dict with
    traced_pixels (used), lookahead_pixels (traced ahead, unused), levels (GPU
    batches) and the render stats).  0 selects the demo's block size /
    interpolation limit / colour threshold.  exact_batches: one batch per
    level with only the needed points (the image is the same bits)."""
    ds = scene if isinstance(scene, DeviceScene) else DeviceScene(scene)
    p, _ = make_params(width, height, spp, depth, screen, seed, order, device)
    ap = _lib.AdaptiveParams()
    ap.block_size, ap.max_interp, ap.min_delta = int(block_size), int(max_interp), float(min_delta)
    ap.exact_batches = 1 if exact_batches else 0
    out = np.zeros((height, width, 3), dtype=np.float32)
    st = RenderStats()
    _lib.check(_lib.lib().pt_render_adaptive(ds.handle, ctypes.byref(p), ctypes.byref(ap), out.ctypes.data,
                                             ctypes.byref(st)))
    info = st.as_dict()
    info.update(traced_pixels=int(ap.traced_pixels), levels=int(ap.levels),
                lookahead_pixels=int(ap.lookahead_pixels))
    return out, info


def prepare(scene: DeviceScene, params: RenderParams) -> None:
    """Load/upload/allocate everything a render with `params` needs."""
    _lib.check(_lib.lib().pt_prepare(scene.handle, ctypes.byref(params)))


def render_device(scene: DeviceScene, params: RenderParams, fb_ptr: int, stream_ptr: int = 0, stats: bool = False):
    """Render into device memory fb_ptr (W*H*3 floats) on stream_ptr
    (synchronous when stats are asked for: they need the kernel timings)."""
    st = RenderStats()
    _lib.check(_lib.lib().pt_render_device(scene.handle, ctypes.byref(params), ctypes.c_void_p(fb_ptr),
                                           ctypes.c_void_p(stream_ptr), ctypes.byref(st) if stats else None))
    return st.as_dict() if stats else None


def render_device_timed(scene: DeviceScene, params: RenderParams, fb_ptr: int, stream_ptr: int = 0) -> None:
    """render_device without a host wait: its kernel timings and counters are
    kept on the device until render_collect (pt_render_device_timed)."""
    _lib.check(_lib.lib().pt_render_device_timed(scene.handle, ctypes.byref(params), ctypes.c_void_p(fb_ptr),
                                                 ctypes.c_void_p(stream_ptr)))


def render_collect(scene: DeviceScene, device: int = 0) -> dict:
    """Summed statistics of the timed renders since the last collect (waits for them)."""
    st = RenderStats()
    _lib.check(_lib.lib().pt_render_collect(scene.handle, int(device), ctypes.byref(st)))
    return st.as_dict()
