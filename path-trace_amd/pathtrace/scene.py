"""Scene-graph API of the reference, mirrored in Python.

Class names, constructor arguments and defaults follow the reference's public
C++ API:

  Sphere(center, r, material)                      include/sphere.h:12
  Plane(normal, d, material) / Plane(normal, pos, material)   include/plane.h:12-13
  Union / Intersection / Difference(a, b)          include/{union,intersection,difference}.h:12
  TransformedObject(matrix, object)                include/object.h:78
  Material(reflect=ColorTexture(1), scatter_coefficient=ColorTexture(1),
           emissive=ColorTexture(0), transmit=ColorTexture(0), ior=1,
           transmit_reflect_coefficient=ColorTexture(0))   include/material.h:18
  ColorTexture, ImageTexture, ImageAlphaTexture, ImageSkyboxTexture,
  ImageSkyboxAlphaTexture, MultiplyTexture, LogTexture,
  MirrorBallSkymapTexture, SphericalCoordinatesSkymapTexture, TransformedTexture

Every float is rounded to float32 at construction, exactly where the C++
constructors would store a `float`.  A scene serialises to the plain-text scene
format (see `to_text`) that the C-ABI loader `pt_scene_from_text`, the CPU oracle
and the reference driver all read; floats travel as hex floats, so every reader
sees the same bits.
"""
from __future__ import annotations

import os
import struct
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np

f32 = np.float32


def _f(v) -> np.float32:
    return f32(v)


def _hex(v) -> str:
    return float(f32(v)).hex()


def vec(v) -> Tuple[np.float32, np.float32, np.float32]:
    if isinstance(v, (int, float, np.floating)):
        return (_f(v), _f(v), _f(v))
    x, y, z = v
    return (_f(x), _f(y), _f(z))


# ----------------------------------------------------------------- matrix ---
class Matrix:
    """3x4 affine matrix, constructor order x00 x10 x20 x30 x01 x11 x21 x31
    x02 x12 x22 x32 (include/transform.h:148-174).  The factory/algebra
    helpers delegate to the product library so their float arithmetic is the
    C++ arithmetic of include/transform.h:207-421."""

    __slots__ = ("m",)

    def __init__(self, *vals):
        if len(vals) == 0:
            vals = (1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1, 0)
        if len(vals) == 1:
            vals = tuple(vals[0])
        if len(vals) != 12:
            raise ValueError("Matrix takes 12 values")
        self.m = tuple(_f(v) for v in vals)

    def __eq__(self, other):
        return isinstance(other, Matrix) and all(
            np.float32(a) == np.float32(b) for a, b in zip(self.m, other.m))

    def __repr__(self):
        return "Matrix(%s)" % ", ".join(repr(float(v)) for v in self.m)

    @staticmethod
    def identity():
        return Matrix()

    @staticmethod
    def translate(x, y=None, z=None):
        if y is None:
            x, y, z = vec(x)
        return Matrix(1, 0, 0, x, 0, 1, 0, y, 0, 0, 1, z)

    @staticmethod
    def scale(x, y=None, z=None):
        if y is None:
            x, y, z = vec(x)
        return Matrix(x, 0, 0, 0, 0, y, 0, 0, 0, 0, z, 0)

    @staticmethod
    def rotate(axis, angle):
        from . import _lib
        return Matrix(_lib.matrix_rotate(vec(axis), float(angle)))

    @staticmethod
    def rotateX(angle):
        return Matrix.rotate((1, 0, 0), angle)

    @staticmethod
    def rotateY(angle):
        return Matrix.rotate((0, 1, 0), angle)

    @staticmethod
    def rotateZ(angle):
        return Matrix.rotate((0, 0, 1), angle)

    def inverse(self):
        from . import _lib
        return Matrix(_lib.matrix_inverse(self.m))

    def concat(self, rt: "Matrix"):
        from . import _lib
        return Matrix(_lib.matrix_concat(self.m, rt.m))

    def apply(self, v):
        x, y, z = vec(v)
        m = self.m
        return ((x * m[0] + y * m[1]) + z * m[2] + m[3],
                (x * m[4] + y * m[5]) + z * m[6] + m[7],
                (x * m[8] + y * m[9]) + z * m[10] + m[11])


def invert(m: Matrix) -> Matrix:
    return m.inverse()


# ----------------------------------------------------------------- images ---
class Image:
    """Refcounted RGBA float image (include/image.h:48-101).  Row 0 is the top
    row, 4 floats per pixel."""

    def __init__(self, data=None, path: Optional[str] = None):
        if path is not None:
            # Image(string fileName): format from the extension (src/image.cpp:49-83)
            from . import _lib
            ext = path.rsplit(".", 1)[-1].lower() if "." in path else ""
            if ext == "png":
                data = _lib.load_png(path)
            elif ext in ("hdr", "pic"):
                data = _lib.load_hdr(path)
            else:
                raise _lib.PtError("can't determine format" if not ext else "invalid format")
        if data is None:
            raise ValueError("Image needs data or a path")
        data = np.ascontiguousarray(data, dtype=np.float32)
        if data.ndim != 3 or data.shape[2] != 4:
            raise ValueError("Image data must be H x W x 4 float32")
        self.data = data

    @property
    def width(self):
        return self.data.shape[1]

    @property
    def height(self):
        return self.data.shape[0]


# --------------------------------------------------------------- textures ---
class Texture:
    kind = "?"

    def children(self) -> List["Texture"]:
        return []

    def transform(self, m: Matrix):  # include/texture.h:19-22
        return None


class ColorTexture(Texture):
    kind = "color"

    def __init__(self, *c):
        if len(c) == 1:
            c = vec(c[0])
        self.color = vec(c)

    def transform(self, m):  # texture.h:51-54
        return ColorTexture(self.color)


class CoordTexture(Texture):
    """Test instrument (not in the reference): colour = lookup coordinate."""
    kind = "coord"


class DeviceTexture(Texture):
    """A user-defined Texture subclass (reference include/texture.h:10-27) given
    as device source (pt_tex_device): `color_body` is the body of
    V3 getColor(V3 p), `value_body` (None = the reference's default mean of
    getColor) the body of float getFloat(V3 p); both read `params` as
    `const float *prm`.  `oracle_slot` names the host function the CPU oracle
    calls for it (oracle_py.register_user_texture, test infrastructure)."""
    kind = "user"

    def __init__(self, color_body: str, params=(), value_body: Optional[str] = None, oracle_slot: int = 0):
        self.color_body = color_body
        self.value_body = value_body
        self.params = [float(v) for v in params]
        self.oracle_slot = int(oracle_slot)


class ImageTexture(Texture):
    kind = "image"

    def __init__(self, image: Image):
        self.image = image


class ImageAlphaTexture(ImageTexture):
    kind = "image_alpha"


class ImageSkyboxTexture(Texture):
    kind = "skybox"

    def __init__(self, top, bottom, left, right, front, back):
        self.faces = [top, bottom, left, right, front, back]


class ImageSkyboxAlphaTexture(ImageSkyboxTexture):
    kind = "skybox_alpha"


class MultiplyTexture(Texture):
    kind = "multiply"

    def __init__(self, factor, t: Texture):
        self.factor = vec(factor)
        self.t = t

    def children(self):
        return [self.t]


class LogTexture(Texture):
    kind = "log"

    def __init__(self, t: Texture):
        self.t = t

    def children(self):
        return [self.t]


class MirrorBallSkymapTexture(LogTexture):
    kind = "mirrorball"


class SphericalCoordinatesSkymapTexture(LogTexture):
    kind = "spherical"


class TransformedTexture(Texture):
    kind = "xform"

    def __init__(self, m: Matrix, t: Texture):
        self.matrix = m
        self.t = t

    def children(self):
        return [self.t]

    def transform(self, m):  # texture.h:86-89
        return TransformedTexture(self.matrix.concat(m), self.t)


def transform_texture(m: Matrix, t: Texture) -> Texture:
    r = t.transform(m)
    return r if r is not None else TransformedTexture(m, t)


# -------------------------------------------------------------- materials ---
class Material:
    def __init__(self, reflect=None, scatter_coefficient=None, emissive=None, transmit=None, ior=1.0,
                 transmit_reflect_coefficient=None):
        self.reflect = reflect if reflect is not None else ColorTexture(1)
        self.scatter_coefficient = scatter_coefficient if scatter_coefficient is not None else ColorTexture(1)
        self.emissive = emissive if emissive is not None else ColorTexture(0)
        self.transmit = transmit if transmit is not None else ColorTexture(0)
        self.ior = _f(ior)
        self.transmit_reflect_coefficient = (transmit_reflect_coefficient if transmit_reflect_coefficient
                                             is not None else ColorTexture(0))

    def textures(self):
        return [self.reflect, self.scatter_coefficient, self.emissive, self.transmit,
                self.transmit_reflect_coefficient]


def transform_material(m: Matrix, mat: Material) -> Material:  # include/material.h:39-42
    return Material(transform_texture(m, mat.reflect), transform_texture(m, mat.scatter_coefficient),
                    transform_texture(m, mat.emissive), transform_texture(m, mat.transmit), mat.ior,
                    transform_texture(m, mat.transmit_reflect_coefficient))


# ---------------------------------------------------------------- objects ---
class Object:
    kind = "?"

    def children(self) -> List["Object"]:
        return []

    def transform(self, m: Matrix):  # include/object.h:15-18
        return None

    def duplicate(self):
        raise NotImplementedError


class Sphere(Object):
    kind = "sphere"

    def __init__(self, center, r, material: Material):
        self.center = vec(center)
        self.r = _f(r)
        self.material = material

    def duplicate(self):
        return Sphere(self.center, self.r, self.material)


class DeviceObject(Object):
    """A user-defined Object subclass (reference include/object.h:10-24) with
    one span per ray, given as device source (pt_object_device): `span_body`
    is the body of bool span(V3 o, V3 d, float &t0, float &t1), `normal_body`
    the body of V3 normal(V3 p); both read `params` as `const float *prm`.
    `oracle_slot` names the host functions the CPU oracle calls for it
    (oracle_py.register_user_object, test infrastructure)."""
    kind = "user"

    def __init__(self, span_body: str, normal_body: str, params, material: Material, oracle_slot: int = 0):
        self.span_body = span_body
        self.normal_body = normal_body
        self.params = [float(v) for v in params]
        self.material = material
        self.oracle_slot = int(oracle_slot)

    def duplicate(self):
        return DeviceObject(self.span_body, self.normal_body, self.params, self.material, self.oracle_slot)


class Plane(Object):
    """Half-space {p : normal.p + d < 0} (src/plane.cpp:23-63).  Plane(n, d, m)
    or Plane(n, point, m) with d = -dot(n, point) (src/plane.cpp:11-14)."""
    kind = "plane"

    def __init__(self, normal, d, material: Material):
        self.normal = vec(normal)
        if isinstance(d, (int, float, np.floating)):
            self.d = _f(d)
        else:
            p = vec(d)
            n = self.normal
            self.d = -((n[0] * p[0] + n[1] * p[1]) + n[2] * p[2])
        self.material = material

    def duplicate(self):
        return Plane(self.normal, self.d, self.material)


class _Binary(Object):
    def __init__(self, a: Object, b: Object):
        self.a, self.b = a, b

    def children(self):
        return [self.a, self.b]

    def duplicate(self):
        return type(self)(self.a.duplicate(), self.b.duplicate())

    def transform(self, m):
        # include/union.h:21, intersection.h:21, difference.h:21 transform `a`
        # twice (the second operand is dropped); kept for drop-in fidelity.
        return type(self)(transform_object(m, self.a), transform_object(m, self.a))


class Union(_Binary):
    kind = "union"


class Intersection(_Binary):
    kind = "intersection"


class Difference(_Binary):
    kind = "difference"


class TransformedObject(Object):
    kind = "xform"

    def __init__(self, m: Matrix, o: Object):
        self.matrix = m
        self.o = o

    def children(self):
        return [self.o]

    def transform(self, m):  # include/object.h:85-88
        return TransformedObject(self.matrix.concat(m), self.o.duplicate())

    def duplicate(self):
        return TransformedObject(self.matrix, self.o.duplicate())


def transform_object(m: Matrix, o: Object) -> Object:  # include/object.h:100-106
    r = o.transform(m)
    return r if r is not None else TransformedObject(m, o.duplicate())


def union_array(objs: Sequence[Object]) -> Object:
    """Balanced union tree, as the reference demo builds its world (src/test.cpp:52-64)."""
    n = len(objs)
    if n == 1:
        return objs[0]
    if n == 2:
        return Union(objs[0], objs[1])
    split = n // 2
    return Union(union_array(objs[:split]), union_array(objs[split:]))


# ---------------------------------------------------------- serialisation ---
class _Registry:
    def __init__(self):
        self.images: Dict[int, Tuple[int, Image]] = {}
        self.tex_lines: List[str] = []
        self.mat_ids: Dict[int, int] = {}
        self.mat_lines: List[str] = []
        self.obj_lines: List[str] = []
        self.n_tex = 0
        self.n_obj = 0

    def image(self, im: Image) -> int:
        key = id(im)
        if key not in self.images:
            self.images[key] = (len(self.images), im)
        return self.images[key][0]

    def texture(self, t: Texture) -> int:
        if isinstance(t, ColorTexture):
            args = " ".join(_hex(c) for c in t.color)
        elif isinstance(t, CoordTexture):
            args = ""
        elif isinstance(t, DeviceTexture):  # the oracle's host function for the slot + the parameters
            args = "%d %d %s" % (t.oracle_slot, len(t.params), " ".join(_hex(v) for v in t.params))
        elif isinstance(t, ImageSkyboxTexture):
            args = " ".join(str(self.image(f)) for f in t.faces)
        elif isinstance(t, ImageTexture):
            args = str(self.image(t.image))
        elif isinstance(t, MultiplyTexture):
            args = " ".join(_hex(c) for c in t.factor) + " %d" % self.texture(t.t)
        elif isinstance(t, TransformedTexture):
            args = " ".join(_hex(c) for c in t.matrix.m) + " %d" % self.texture(t.t)
        elif isinstance(t, LogTexture):  # log / mirrorball / spherical
            args = str(self.texture(t.t))
        else:
            raise TypeError("cannot serialise texture %r" % (t,))
        tid = self.n_tex
        self.n_tex += 1
        self.tex_lines.append(("tex %d %s %s" % (tid, t.kind, args)).rstrip())
        return tid

    def material(self, m: Material) -> int:
        key = id(m)
        if key not in self.mat_ids:
            ids = [self.texture(t) for t in m.textures()]
            mid = len(self.mat_ids)
            self.mat_ids[key] = mid
            self.mat_lines.append("mat %d %d %d %d %d %s %d" % (mid, ids[0], ids[1], ids[2], ids[3],
                                                                 _hex(m.ior), ids[4]))
        return self.mat_ids[key]

    def obj(self, o: Object) -> int:
        if isinstance(o, Sphere):
            args = "%s %s %s %s %d" % (*(_hex(c) for c in o.center), _hex(o.r), self.material(o.material))
        elif isinstance(o, Plane):
            args = "%s %s %s %s %d" % (*(_hex(c) for c in o.normal), _hex(o.d), self.material(o.material))
        elif isinstance(o, DeviceObject):  # the oracle's host functions for the slot, the material, the parameters
            args = "%d %d %d %s" % (o.oracle_slot, self.material(o.material), len(o.params),
                                    " ".join(_hex(v) for v in o.params))
        elif isinstance(o, _Binary):
            a = self.obj(o.a)
            b = self.obj(o.b)
            args = "%d %d" % (a, b)
        elif isinstance(o, TransformedObject):
            c = self.obj(o.o)
            args = " ".join(_hex(v) for v in o.matrix.m) + " %d" % c
        else:
            raise TypeError("cannot serialise object %r" % (o,))
        oid = self.n_obj
        self.n_obj += 1
        self.obj_lines.append("obj %d %s %s" % (oid, o.kind, args))
        return oid


def to_text(root: Object, image_dir: Optional[str] = None) -> str:
    """Serialise a scene graph to the plain-text scene format.  Images are
    written as raw little-endian RGBA32F files into `image_dir`."""
    reg = _Registry()
    rid = reg.obj(root)
    lines = []
    for _, (iid, im) in sorted(reg.images.items(), key=lambda kv: kv[1][0]):
        if image_dir is None:
            raise ValueError("scene has images: pass image_dir")
        os.makedirs(image_dir, exist_ok=True)
        path = os.path.join(image_dir, "img%d.rgba32f" % iid)
        im.data.astype("<f4").tofile(path)
        lines.append("image %d raw %d %d %s" % (iid, im.width, im.height, path))
    lines += reg.tex_lines + reg.mat_lines + reg.obj_lines
    lines.append("root %d" % rid)
    return "\n".join(lines) + "\n"


def count_primitives(root: Object) -> int:
    if isinstance(root, (Sphere, Plane)):
        return 1
    return sum(count_primitives(c) for c in root.children())
