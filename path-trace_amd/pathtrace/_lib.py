"""ctypes binding of libpt.so (include/pt/pt.h).  The product path: every
render goes through this C ABI into the HIP megakernel; there is no CPU
fallback -- if the library or a GPU is missing, calls raise."""
from __future__ import annotations

import ctypes
import os
from typing import Optional, Sequence

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.normpath(os.path.join(HERE, "..", "lib", "libpt.so"))

PT_ORDER_FAST = 0
PT_ORDER_REFERENCE = 1
PT_CSG_UNION, PT_CSG_INTERSECTION, PT_CSG_DIFFERENCE = 0, 1, 2


class PtError(RuntimeError):
    pass


class RenderParams(ctypes.Structure):
    _fields_ = [("width", ctypes.c_int), ("height", ctypes.c_int), ("spp", ctypes.c_int), ("depth", ctypes.c_int),
                ("screen_w", ctypes.c_float), ("screen_h", ctypes.c_float), ("screen_dist", ctypes.c_float),
                ("seed", ctypes.c_uint64), ("order", ctypes.c_int), ("device", ctypes.c_int),
                ("pixels", ctypes.POINTER(ctypes.c_int32)), ("npixels", ctypes.c_int64),
                ("max_buffer_bytes", ctypes.c_int64), ("grid_width", ctypes.c_int),
                ("sample_begin", ctypes.c_int), ("sum_only", ctypes.c_int)]


class AdaptiveParams(ctypes.Structure):
    _fields_ = [("block_size", ctypes.c_int), ("max_interp", ctypes.c_int), ("min_delta", ctypes.c_float),
                ("traced_pixels", ctypes.c_int64), ("levels", ctypes.c_int), ("exact_batches", ctypes.c_int),
                ("lookahead_pixels", ctypes.c_int64)]


class TraceParams(ctypes.Structure):
    _fields_ = [("spp", ctypes.c_int), ("depth", ctypes.c_int), ("seed", ctypes.c_uint64), ("order", ctypes.c_int),
                ("device", ctypes.c_int), ("sample_begin", ctypes.c_int), ("max_buffer_bytes", ctypes.c_int64),
                ("ray_begin", ctypes.c_int64)]


class RenderStats(ctypes.Structure):
    _fields_ = [("kernel_ms", ctypes.c_double), ("reduce_ms", ctypes.c_double), ("launches", ctypes.c_uint64),
                ("samples", ctypes.c_uint64), ("queries", ctypes.c_uint64), ("leaf_queries", ctypes.c_uint64),
                ("attempts", ctypes.c_uint64), ("rounds", ctypes.c_uint64), ("sphere_tests", ctypes.c_uint64),
                ("sphere_hits", ctypes.c_uint64), ("plane_tests", ctypes.c_uint64),
                ("slow_queries", ctypes.c_uint64), ("dark_queries", ctypes.c_uint64),
                ("mid_queries", ctypes.c_uint64), ("wave_ms", ctypes.c_double)]

    def as_dict(self):
        return {k: getattr(self, k) for k, _ in self._fields_}


# every symbol include/pt/pt.h declares, with its ctypes signature
_P = ctypes.c_void_p
_I = ctypes.c_int
_F = ctypes.c_float
_FP = ctypes.POINTER(ctypes.c_float)
SIGNATURES = {
    "pt_scene_create": (_P, []),
    "pt_scene_destroy": (None, [_P]),
    "pt_last_error": (ctypes.c_char_p, []),
    "pt_version": (ctypes.c_char_p, []),
    "pt_image_load_hdr": (_I, [_P, ctypes.c_char_p]),
    "pt_image_load_png": (_I, [_P, ctypes.c_char_p]),
    "pt_image_load": (_I, [_P, ctypes.c_char_p]),
    "pt_image_from_rgba32f": (_I, [_P, _P, _I, _I]),
    "pt_hdr_read": (_I, [ctypes.c_char_p, _P, ctypes.POINTER(_I), ctypes.POINTER(_I)]),
    "pt_png_read": (_I, [ctypes.c_char_p, _P, ctypes.POINTER(_I), ctypes.POINTER(_I)]),
    "pt_tex_color": (_I, [_P, _F, _F, _F]),
    "pt_tex_image": (_I, [_P, _I]),
    "pt_tex_image_alpha": (_I, [_P, _I]),
    "pt_tex_skybox": (_I, [_P, _I, _I, _I, _I, _I, _I]),
    "pt_tex_skybox_alpha": (_I, [_P, _I, _I, _I, _I, _I, _I]),
    "pt_tex_multiply": (_I, [_P, _F, _F, _F, _I]),
    "pt_tex_log": (_I, [_P, _I]),
    "pt_tex_mirrorball": (_I, [_P, _I]),
    "pt_tex_spherical": (_I, [_P, _I]),
    "pt_tex_transformed": (_I, [_P, _FP, _I]),
    "pt_tex_coord": (_I, [_P]),
    "pt_tex_device": (_I, [_P, ctypes.c_char_p, ctypes.c_char_p, ctypes.POINTER(ctypes.c_float), _I]),
    "pt_object_device": (_I, [_P, ctypes.c_char_p, ctypes.c_char_p, ctypes.POINTER(ctypes.c_float), _I, _I]),
    "pt_material": (_I, [_P, _I, _I, _I, _I, _F, _I]),
    "pt_sphere": (_I, [_P, _F, _F, _F, _F, _I]),
    "pt_plane": (_I, [_P, _F, _F, _F, _F, _I]),
    "pt_plane_through": (_I, [_P, _F, _F, _F, _F, _F, _F, _I]),
    "pt_csg": (_I, [_P, _I, _I, _I]),
    "pt_transformed": (_I, [_P, _FP, _I]),
    "pt_set_root": (_I, [_P, _I]),
    "pt_scene_from_text": (_I, [_P, ctypes.c_char_p]),
    "pt_matrix_rotate": (None, [_FP, ctypes.c_double, _FP]),
    "pt_matrix_inverse": (_I, [_FP, _FP]),
    "pt_matrix_concat": (None, [_FP, _FP, _FP]),
    "pt_render": (_I, [_P, ctypes.POINTER(RenderParams), _P, ctypes.POINTER(RenderStats)]),
    "pt_render_device": (_I, [_P, ctypes.POINTER(RenderParams), _P, _P, ctypes.POINTER(RenderStats)]),
    "pt_render_device_timed": (_I, [_P, ctypes.POINTER(RenderParams), _P, _P]),
    "pt_render_collect": (_I, [_P, _I, ctypes.POINTER(RenderStats)]),
    "pt_call_profile": (_I, [ctypes.POINTER(ctypes.c_double), _I]),
    "pt_rank_pixels": (_I, [_I, _I, _I, _I, _I, _P, ctypes.c_int64, ctypes.POINTER(ctypes.c_int64)]),
    "pt_render_adaptive": (_I, [_P, ctypes.POINTER(RenderParams), ctypes.POINTER(AdaptiveParams), _P,
                                ctypes.POINTER(RenderStats)]),
    "pt_trace_rays": (_I, [_P, ctypes.POINTER(TraceParams), _P, ctypes.c_int64, _P, ctypes.POINTER(RenderStats)]),
    "pt_trace_compile": (_I, [_P, _I]),
    "pt_prepare": (_I, [_P, ctypes.POINTER(RenderParams)]),
    "pt_scene_compile": (_I, [_P, _I]),
    "pt_scene_set_occupancy": (_I, [_P, _I]),
    "pt_scene_set_fast_spine": (_I, [_P, _I]),
    "pt_scene_set_lane_walk": (_I, [_P, _I]),
    "pt_scene_set_split": (_I, [_P, _I]),
    "pt_scene_set_lane_scatter": (_I, [_P, _I]),
    "pt_scene_kernel_key": (ctypes.c_char_p, [_P, _I]),
    "pt_selftest_math": (_I, [_I, ctypes.c_uint64, ctypes.c_uint64, _P]),
    "pt_selftest_libm": (_I, [_I, _P, ctypes.c_int64, _P]),
    "pt_query_spans": (_I, [_P, _I, _P, ctypes.c_int64, _I, _P, _P, _I]),
    "pt_tex_eval": (_I, [_P, _I, _P, ctypes.c_int64, _P, _P, _I]),
    "pt_query_compile": (_I, [_P, _I, _I]),
    "pt_write_hdr": (_I, [ctypes.c_char_p, _P, _I, _I]),
    "pt_write_bmp": (_I, [ctypes.c_char_p, _P, _I, _I, _I]),
}

_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise PtError("libpt.so not built: run `python path-trace_amd/build_ext.py` (%s)" % LIB_PATH)
        # libpt binds the process's HIP runtime (soname libamdhip64.so.7).  torch
        # loads its own copy under another file name; loading torch first makes
        # libpt share it, so torch's device pointers/streams are valid in libpt
        # and the process holds one runtime, not two competing for the device.
        try:
            import torch  # noqa: F401
        except ImportError:
            pass
        L = ctypes.CDLL(LIB_PATH)
        for name, (res, args) in SIGNATURES.items():
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        _lib = L
    return _lib


def check(rc: int) -> int:
    if rc < 0:
        raise PtError(lib().pt_last_error().decode() or ("pt error %d" % rc))
    return rc


def _f12(vals) -> ctypes.Array:
    return (ctypes.c_float * 12)(*[float(v) for v in vals])


def matrix_rotate(axis, angle: float):
    out = (ctypes.c_float * 12)()
    lib().pt_matrix_rotate((ctypes.c_float * 3)(*[float(a) for a in axis]), float(angle), out)
    return [np.float32(v) for v in out]


def matrix_inverse(m):
    out = (ctypes.c_float * 12)()
    check(lib().pt_matrix_inverse(_f12(m), out))
    return [np.float32(v) for v in out]


def matrix_concat(a, b):
    out = (ctypes.c_float * 12)()
    lib().pt_matrix_concat(_f12(a), _f12(b), out)
    return [np.float32(v) for v in out]


def selftest_math(n: int = 1 << 26, seed: int = 1, device: int = 0):
    out = np.zeros(3, dtype=np.uint64)
    check(lib().pt_selftest_math(device, n, seed, out.ctypes.data))
    return dict(zip(["sqrt", "div", "normalize"], [int(v) for v in out]))


def _read(fn, path: str) -> np.ndarray:
    w = ctypes.c_int(0)
    h = ctypes.c_int(0)
    check(fn(path.encode(), None, ctypes.byref(w), ctypes.byref(h)))
    out = np.zeros((h.value, w.value, 4), dtype=np.float32)
    check(fn(path.encode(), out.ctypes.data, ctypes.byref(w), ctypes.byref(h)))
    return out


def load_hdr(path: str) -> np.ndarray:
    """Radiance HDR decode (reference src/image.cpp:83-324): h x w x RGBA float32."""
    return _read(lib().pt_hdr_read, path)


def load_png(path: str) -> np.ndarray:
    """PNG decode as the reference's Image(fileName) (src/image.cpp:60-79): h x w x RGBA float32."""
    return _read(lib().pt_png_read, path)


def write_hdr(path: str, rgb: np.ndarray) -> None:
    rgb = np.ascontiguousarray(rgb, dtype=np.float32)
    h, w = rgb.shape[:2]
    check(lib().pt_write_hdr(path.encode(), rgb.ctypes.data, w, h))


def write_bmp(path: str, rgb: np.ndarray, count: int = 1) -> None:
    rgb = np.ascontiguousarray(rgb, dtype=np.float32)
    h, w = rgb.shape[:2]
    check(lib().pt_write_bmp(path.encode(), rgb.ctypes.data, w, h, count))


def selftest_libm(ops, device: int = 0):
    """The device's restated atan2f / asinf / logf (pt_selftest_libm) on operand
    pairs ops (n x 2 float32: y, x): returns n x 3 (atan2f(y, x), asinf(y), logf(x))."""
    import numpy as np
    ops = np.ascontiguousarray(ops, dtype=np.float32).reshape(-1, 2)
    out = np.zeros((len(ops), 3), dtype=np.float32)
    check(lib().pt_selftest_libm(device, ops.ctypes.data, len(ops), out.ctypes.data))
    return out
