"""TEST INFRASTRUCTURE ONLY -- Python access to the CPU oracle
(oracle/build/liboracle.so, a restatement of the reference hot path) and to
the reference driver (oracle/_ref/ptref, the unmodified reference sources).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import
this module; the product (path-trace_amd/) never does.
"""
from __future__ import annotations

import ctypes
import json
import os
import subprocess
import tempfile
from typing import List, Optional, Sequence

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "build", "liboracle.so")
REF_PATH = os.path.join(HERE, "_ref", "ptref")

ORDER_REFERENCE = 0
ORDER_FAST = 1

STAT_NAMES = ["queries", "sphere_tests", "sphere_hits", "plane_tests", "merge_steps", "shaded",
              "refract_children", "scatter_children", "attempts", "draws", "leaf_children",
              # texture evaluations by class (oracle.cpp TexCount)
              "tex_xform", "tex_multiply", "tex_image", "tex_spherical", "tex_mirrorball", "tex_skybox", "tex_log"]

_lib = None


def build(ref: bool = False) -> None:
    """Compile the oracle (and, when /root/reference exists, the reference driver)."""
    subprocess.check_call(["make", "-s", "-C", HERE, "all"])
    if ref and os.path.isdir("/root/reference"):
        subprocess.check_call(["make", "-s", "-C", HERE, "ref"])


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = ctypes.CDLL(LIB_PATH)
        L.oracle_last_error.restype = ctypes.c_char_p
        L.oracle_render.restype = ctypes.c_int
        L.oracle_render.argtypes = [ctypes.c_char_p, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                    ctypes.c_float, ctypes.c_float, ctypes.c_float, ctypes.c_uint64,
                                    ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                    ctypes.c_void_p, ctypes.c_void_p]
        L.oracle_spans.restype = ctypes.c_int
        L.oracle_spans.argtypes = [ctypes.c_char_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p,
                                   ctypes.c_int64, ctypes.POINTER(ctypes.c_int64)]
        L.oracle_tex_eval.restype = ctypes.c_int
        L.oracle_tex_eval.argtypes = [ctypes.c_char_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p]
        C = ctypes
        L.oracle_render_gw.restype = C.c_int
        L.oracle_render_gw.argtypes = [C.c_char_p, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.c_float, C.c_float,
                                       C.c_float, C.c_uint64, C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_int,
                                       C.c_void_p, C.c_void_p]
        L.oracle_render_adaptive.restype = C.c_int
        L.oracle_render_adaptive.argtypes = [C.c_char_p, C.c_int, C.c_int, C.c_int, C.c_int, C.c_float, C.c_float,
                                             C.c_float, C.c_uint64, C.c_int, C.c_int, C.c_float, C.c_int, C.c_int,
                                             C.c_void_p, C.c_void_p]
        L.oracle_trace_rays.restype = C.c_int
        L.oracle_trace_rays.argtypes = [C.c_char_p, C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_uint64, C.c_int,
                                        C.c_int64, C.c_int, C.c_int, C.c_void_p]
        L.oracle_register_user_object.restype = ctypes.c_int
        L.oracle_register_user_object.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p]
        L.oracle_register_user_texture.restype = ctypes.c_int
        L.oracle_register_user_texture.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p]
        L.oracle_kat.restype = ctypes.c_int
        L.oracle_kat.argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.POINTER(ctypes.c_int64)]
        _lib = L
    return _lib


def render(scene_text: str, W: int, H: int, spp: int, depth: int, screen=None, seed: int = 0x5EED,
           pixels: Optional[Sequence[int]] = None, threads: int = 0, order: int = ORDER_REFERENCE,
           per_sample: bool = False, stats: bool = False):
    """Per-pixel mean radiance (npx x 3 float32), or per-sample (npx x spp x 3)."""
    sw, sh, dist = screen if screen is not None else (float(W), float(H), float(2 * min(W, H)))
    L = lib()
    px = None if pixels is None else np.ascontiguousarray(np.asarray(pixels, dtype=np.int32))
    npx = W * H if px is None else len(px)
    out = np.zeros((npx, spp, 3) if per_sample else (npx, 3), dtype=np.float32)
    st = np.zeros(24, dtype=np.uint64)
    if threads <= 0:
        threads = os.cpu_count() or 1
    rc = L.oracle_render(scene_text.encode(), W, H, spp, depth, sw, sh, dist, seed,
                         None if px is None else px.ctypes.data, npx, threads, order, int(per_sample),
                         out.ctypes.data, st.ctypes.data)
    if rc != 0:
        raise RuntimeError("oracle_render: " + L.oracle_last_error().decode())
    if stats:
        return out, dict(zip(STAT_NAMES, [int(v) for v in st[:len(STAT_NAMES)]]))
    return out


def render_gw(scene_text: str, W: int, H: int, gw: int, pixels, spp: int, depth: int, screen=None,
              seed: int = 0x5EED, threads: int = 0, order: int = ORDER_REFERENCE):
    """Per-pixel means for grid indices p = py * gw + px (gw >= W)."""
    sw, sh, dist = screen if screen is not None else (float(W), float(H), float(2 * min(W, H)))
    L = lib()
    px = np.ascontiguousarray(np.asarray(pixels, dtype=np.int32))
    out = np.zeros((len(px), 3), dtype=np.float32)
    rc = L.oracle_render_gw(scene_text.encode(), W, H, gw, spp, depth, sw, sh, dist, seed, px.ctypes.data, len(px),
                            threads or (os.cpu_count() or 1), order, 0, out.ctypes.data, None)
    if rc != 0:
        raise RuntimeError("oracle_render_gw: " + L.oracle_last_error().decode())
    return out


def render_adaptive(scene_text: str, W: int, H: int, spp: int, depth: int, block: int, max_interp: int,
                    min_delta: float = 0.003, screen=None, seed: int = 0x5EED, threads: int = 0,
                    order: int = ORDER_REFERENCE):
    """RenderBlock restated depth-first (oracle.cpp AdaptiveBlock): (H x W x 3, traced pixel count)."""
    sw, sh, dist = screen if screen is not None else (float(W), float(H), float(2 * min(W, H)))
    L = lib()
    out = np.zeros((H, W, 3), dtype=np.float32)
    traced = np.zeros(1, dtype=np.uint64)
    rc = L.oracle_render_adaptive(scene_text.encode(), W, H, spp, depth, sw, sh, dist, seed, block, max_interp,
                                  min_delta, threads or (os.cpu_count() or 1), order, out.ctypes.data,
                                  traced.ctypes.data)
    if rc != 0:
        raise RuntimeError("oracle_render_adaptive: " + L.oracle_last_error().decode())
    return out, int(traced[0])


def trace_rays(scene_text: str, rays: np.ndarray, spp: int, depth: int, seed: int = 0x5EED, sample_begin: int = 0,
               threads: int = 0, order: int = ORDER_REFERENCE, ray_begin: int = 0):
    """traceRay per caller ray (n x 7: origin, direction, strength): the mean
    of spp samples keyed (seed, ray, sample) -- pt_trace_rays' restatement."""
    r = np.ascontiguousarray(rays, dtype=np.float32).reshape(-1, 7)
    out = np.zeros((len(r), 3), dtype=np.float32)
    rc = lib().oracle_trace_rays(scene_text.encode(), r.ctypes.data, len(r), spp, depth, seed, sample_begin,
                                 ray_begin, threads or (os.cpu_count() or 1), order, out.ctypes.data)
    if rc != 0:
        raise RuntimeError("oracle_trace_rays: " + lib().oracle_last_error().decode())
    return out


def ref_trace_rays(scene_text: str, rays: np.ndarray, spp: int, depth: int, seed: int = 0x5EED,
                   threads: int = 0):
    """The same from the unmodified reference (ptref "rays" mode:
    PathTrace::traceRay<PtSampleEngine> per (ray, sample), summed in order)."""
    r = np.ascontiguousarray(rays, dtype=np.float32).reshape(-1, 7)
    with tempfile.TemporaryDirectory() as td:
        sp = os.path.join(td, "scene.txt")
        with open(sp, "w") as f:
            f.write(scene_text)
        rp = os.path.join(td, "rays.bin")
        r.tofile(rp)
        op = os.path.join(td, "out.bin")
        _ref(["rays", sp, rp, str(spp), str(depth), str(seed), str(threads or (os.cpu_count() or 1)), op])
        return np.fromfile(op, dtype=np.float32).reshape(len(r), 3)


def _parse_spans(buf: bytes, n: int):
    res = []
    pos = 0
    for _ in range(n):
        c = int(np.frombuffer(buf, dtype=np.int32, count=1, offset=pos)[0])
        pos += 4
        spans = []
        for _ in range(c):
            a = np.frombuffer(buf, dtype=np.float32, count=4, offset=pos)
            m0 = int(np.frombuffer(buf, dtype=np.int32, count=1, offset=pos + 16)[0])
            b = np.frombuffer(buf, dtype=np.float32, count=4, offset=pos + 20)
            m1 = int(np.frombuffer(buf, dtype=np.int32, count=1, offset=pos + 36)[0])
            pos += 40
            spans.append((a.copy(), m0, b.copy(), m1))
        res.append(spans)
    return res


def spans(scene_text: str, rays: np.ndarray):
    rays = np.ascontiguousarray(rays, dtype=np.float32).reshape(-1, 6)
    cap = 1 << 24
    buf = ctypes.create_string_buffer(cap)
    written = ctypes.c_int64(0)
    rc = lib().oracle_spans(scene_text.encode(), rays.ctypes.data, len(rays), buf, cap, ctypes.byref(written))
    if rc != 0:
        raise RuntimeError("oracle_spans: " + lib().oracle_last_error().decode())
    return _parse_spans(buf.raw[:written.value], len(rays))


def kat() -> np.ndarray:
    out = np.zeros(1 << 16, dtype=np.uint32)
    written = ctypes.c_int64(0)
    rc = lib().oracle_kat(out.ctypes.data, len(out), ctypes.byref(written))
    if rc != 0:
        raise RuntimeError("oracle_kat failed")
    return out[:written.value].copy()


# ------------------------------------------------------- reference driver ---
def ref_available() -> bool:
    return os.path.exists(REF_PATH)


def _ref(args: List[str]) -> str:
    r = subprocess.run([REF_PATH] + args, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError("ptref %s failed: %s" % (args[0], r.stderr))
    return r.stdout


def ref_render(scene_text: str, W: int, H: int, spp: int, depth: int, screen=None, seed: int = 0x5EED,
               pixels: Optional[Sequence[int]] = None, threads: int = 0, per_sample: bool = False,
               info: bool = False):
    sw, sh, dist = screen if screen is not None else (float(W), float(H), float(2 * min(W, H)))
    if threads <= 0:
        threads = os.cpu_count() or 1
    with tempfile.TemporaryDirectory() as td:
        sp = os.path.join(td, "scene.txt")
        with open(sp, "w") as f:
            f.write(scene_text)
        if pixels is None:
            pxarg = "all"
            npx = W * H
        else:
            pxarg = os.path.join(td, "px.bin")
            np.asarray(pixels, dtype=np.int32).tofile(pxarg)
            npx = len(pixels)
        op = os.path.join(td, "out.bin")
        out = _ref(["render", sp, str(W), str(H), str(spp), str(depth), float(sw).hex(), float(sh).hex(),
                    float(dist).hex(), str(seed), pxarg, str(threads), str(int(per_sample)), op])
        res = np.fromfile(op, dtype=np.float32)
    res = res.reshape((npx, spp, 3) if per_sample else (npx, 3))
    if info:
        return res, json.loads(out.strip().splitlines()[-1])
    return res


def register_user_object(slot: int, span_fn: int, normal_fn: int) -> None:
    """Test infrastructure: the host functions (addresses of
    int span(const float *o, const float *d, const float *prm, float *t01) and
    void normal(const float *p, const float *prm, float *n)) the oracle calls
    for `obj <id> user <slot> ...` records (pathtrace.scene.DeviceObject)."""
    if lib().oracle_register_user_object(int(slot), span_fn, normal_fn) != 0:
        raise RuntimeError("oracle_register_user_object: null function")


def register_user_texture(slot: int, color_fn: int, value_fn: int = 0) -> None:
    """Test infrastructure: the host functions (addresses of
    void color(const float *p, const float *prm, float *out) and, optionally,
    float value(const float *p, const float *prm)) the oracle calls for
    `tex <id> user <slot> ...` records (pathtrace.scene.DeviceTexture)."""
    if lib().oracle_register_user_texture(int(slot), color_fn, value_fn or None) != 0:
        raise RuntimeError("oracle_register_user_texture: null color function")


def tex_eval(scene_text: str, points: np.ndarray):
    """getColor / getFloat of every texture of the scene (file order) at each
    point: (ntex, npts, 4) float32 r g b value."""
    import re
    pts = np.ascontiguousarray(points, dtype=np.float32).reshape(-1, 3)
    ntex = len(re.findall(r"^tex ", scene_text, flags=re.M))
    out = np.zeros((ntex, len(pts), 4), dtype=np.float32)
    if lib().oracle_tex_eval(scene_text.encode(), pts.ctypes.data, len(pts), out.ctypes.data) != 0:
        raise RuntimeError("oracle_tex_eval: " + lib().oracle_last_error().decode())
    return out


def ref_tex_eval(scene_text: str, points: np.ndarray):
    """The same from the unmodified reference (ptref "tex" mode)."""
    import re
    pts = np.ascontiguousarray(points, dtype=np.float32).reshape(-1, 3)
    ntex = len(re.findall(r"^tex ", scene_text, flags=re.M))
    with tempfile.TemporaryDirectory() as td:
        sp = os.path.join(td, "scene.txt")
        with open(sp, "w") as f:
            f.write(scene_text)
        pp = os.path.join(td, "pts.bin")
        pts.tofile(pp)
        op = os.path.join(td, "out.bin")
        _ref(["tex", sp, pp, op])
        return np.fromfile(op, dtype=np.float32).reshape(ntex, len(pts), 4)


def ref_spans(scene_text: str, rays: np.ndarray):
    rays = np.ascontiguousarray(rays, dtype=np.float32).reshape(-1, 6)
    with tempfile.TemporaryDirectory() as td:
        sp = os.path.join(td, "scene.txt")
        with open(sp, "w") as f:
            f.write(scene_text)
        rp = os.path.join(td, "rays.bin")
        rays.tofile(rp)
        op = os.path.join(td, "out.bin")
        _ref(["spans", sp, rp, op])
        with open(op, "rb") as f:
            buf = f.read()
    return _parse_spans(buf, len(rays))


def ref_kat() -> np.ndarray:
    with tempfile.TemporaryDirectory() as td:
        op = os.path.join(td, "kat.bin")
        _ref(["kat", op])
        return np.fromfile(op, dtype=np.uint32)


def ref_hdr(path: str):
    """Reference HDR loader + writeHDR: (rgba float32 HxWx4, rewritten bytes)."""
    with tempfile.TemporaryDirectory() as td:
        a = os.path.join(td, "px.bin")
        b = os.path.join(td, "re.hdr")
        info = json.loads(_ref(["hdr", path, a, b]).strip().splitlines()[-1])
        px = np.fromfile(a, dtype=np.float32).reshape(info["h"], info["w"], 4)
        with open(b, "rb") as f:
            return px, f.read()


def ref_write_hdr(rgb: np.ndarray) -> bytes:
    rgb = np.ascontiguousarray(rgb, dtype=np.float32)
    h, w = rgb.shape[:2]
    with tempfile.TemporaryDirectory() as td:
        a = os.path.join(td, "rgb.bin")
        b = os.path.join(td, "o.hdr")
        rgb.tofile(a)
        _ref(["writehdr", str(w), str(h), a, b])
        with open(b, "rb") as f:
            return f.read()
