/*
 * PathTrace.hpp -- C++ host facade over the C ABI (pt.h) that mirrors the
 * reference's scene API (namespace PathTrace of programmerjake/path-trace),
 * so reference scene-building code compiles against it unchanged:
 *
 *   Vector3D / Color                 include/vector3d.h:36-162, include/color.h
 *   Matrix                           include/transform.h:16-421 (float arithmetic via pt_matrix_*)
 *   Image, MutableImage              include/image.h:48-212 (HDR load / writeHDR)
 *   Texture + 11 subclasses          include/texture.h, image_texture.h, filter_texture.h,
 *                                    transform_texture.h
 *   Material                         include/material.h:10-43
 *   Object, Sphere, Plane, Union,
 *   Intersection, Difference,
 *   TransformedObject, transform()   include/object.h, sphere.h, plane.h, union.h, ...
 *   Ray, Span, SpanIterator          include/ray.h, include/span.h:12-171
 *   Object::makeSpanIterator(),      the query virtuals, served by the device
 *   Texture::getColor / getFloat     (pt_query_spans / pt_tex_eval)
 *   unionArray                       src/test.cpp:52-64
 *
 * What differs is the last step: instead of world->makeSpanIterator() and a
 * per-pixel tracePixel<T> loop (include/path-trace.h:187-201, src/test.cpp:
 * 441-465), a `Renderer` flattens the object graph through the C ABI once and
 * renders whole frames / pixel lists on the GPU.  Each class carries the
 * `flatten` hook SURVEY.md s8(b) calls for.  Ownership follows the reference:
 * composites own their children, materials own their textures, objects do
 * not own materials.  Errors surface as the reference's exception types
 * (std::domain_error for a singular matrix, ImageLoadError / ImageStoreError)
 * or PathTrace::DeviceError for device / compile failures.
 *
 * Header-only, C++11.  Link with libpt.so.
 */
#ifndef PT_PATHTRACE_HPP
#define PT_PATHTRACE_HPP

#include <algorithm>
#include <cctype>
#include <chrono>
#include <cmath>
#include <condition_variable>
#include <exception>
#include <map>
#include <mutex>
#include <thread>
#include <memory>
#include <stdexcept>
#include <string>
#include <vector>

#include "pt.h"

namespace PathTrace
{

/* ---------------------------------------------------------------- errors -- */
class ImageLoadError : public std::runtime_error
{
public:
    explicit ImageLoadError(const std::string &msg) : std::runtime_error(msg) {}
};
class ImageStoreError : public std::runtime_error
{
public:
    explicit ImageStoreError(const std::string &msg) : std::runtime_error(msg) {}
};
class DeviceError : public std::runtime_error
{
public:
    int code;
    DeviceError(int code, const std::string &msg) : std::runtime_error(msg), code(code) {}
};

inline int ptCheck(int rc)
{
    if (rc >= 0)
        return rc;
    std::string msg = pt_last_error();
    if (rc == PT_ERR_MATH)
        throw std::domain_error(msg);
    if (rc == PT_ERR_IO)
        throw ImageLoadError(msg);
    throw DeviceError(rc, msg);
}

/* -------------------------------------------------------------- Vector3D -- */
class Vector3D
{
public:
    float x, y, z;
    Vector3D() : x(0), y(0), z(0) {}
    Vector3D(float x, float y, float z) : x(x), y(y), z(z) {}
    Vector3D(float v) : x(v), y(v), z(v) {}
    friend Vector3D operator+(const Vector3D &l, const Vector3D &r) { return Vector3D(l.x + r.x, l.y + r.y, l.z + r.z); }
    friend Vector3D operator-(const Vector3D &l, const Vector3D &r) { return Vector3D(l.x - r.x, l.y - r.y, l.z - r.z); }
    friend Vector3D operator*(const Vector3D &l, const Vector3D &r) { return Vector3D(l.x * r.x, l.y * r.y, l.z * r.z); }
    friend Vector3D operator/(const Vector3D &l, const Vector3D &r) { return Vector3D(l.x / r.x, l.y / r.y, l.z / r.z); }
    friend Vector3D operator/(const Vector3D &l, float r) { return Vector3D(l.x / r, l.y / r, l.z / r); }
    friend Vector3D operator*(const Vector3D &l, float r) { return Vector3D(l.x * r, l.y * r, l.z * r); }
    friend Vector3D operator*(float l, const Vector3D &r) { return r * l; }
    Vector3D operator-() const { return Vector3D(-x, -y, -z); }
    friend bool operator==(const Vector3D &l, const Vector3D &r) { return l.x == r.x && l.y == r.y && l.z == r.z; }
    friend bool operator!=(const Vector3D &l, const Vector3D &r) { return !(l == r); }
    Vector3D &operator+=(const Vector3D &r) { return *this = *this + r; }
    Vector3D &operator-=(const Vector3D &r) { return *this = *this - r; }
    Vector3D &operator*=(const Vector3D &r) { return *this = *this * r; }
    Vector3D &operator/=(const Vector3D &r) { return *this = *this / r; }
    Vector3D &operator*=(float r) { return *this = *this * r; }
    Vector3D &operator/=(float r) { return *this = *this / r; }
};

/* same evaluation order as include/vector3d.h:121-141 */
inline float dot(const Vector3D &l, const Vector3D &r)
{
    Vector3D v = l * r;
    return v.x + v.y + v.z;
}
inline float abs_squared(const Vector3D &v) { return dot(v, v); }
inline float abs(const Vector3D &v) { return std::sqrt(abs_squared(v)); }
inline Vector3D normalize(const Vector3D &v)
{
    float m = abs(v);
    return v / (m == 0 ? 1.0f : m);
}
inline Vector3D cross(const Vector3D &a, const Vector3D &b)
{
    return Vector3D(a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x);
}

typedef Vector3D Color;

/* ---------------------------------------------------------------- Matrix -- */
class Matrix
{
public:
    /* constructor order of include/transform.h:148-174 */
    float x00, x10, x20, x30, x01, x11, x21, x31, x02, x12, x22, x32;
    Matrix() : x00(1), x10(0), x20(0), x30(0), x01(0), x11(1), x21(0), x31(0), x02(0), x12(0), x22(1), x32(0) {}
    Matrix(float x00, float x10, float x20, float x30, float x01, float x11, float x21, float x31, float x02,
           float x12, float x22, float x32)
        : x00(x00), x10(x10), x20(x20), x30(x30), x01(x01), x11(x11), x21(x21), x31(x31), x02(x02), x12(x12),
          x22(x22), x32(x32)
    {
    }
    explicit Matrix(const float m[12])
        : Matrix(m[0], m[1], m[2], m[3], m[4], m[5], m[6], m[7], m[8], m[9], m[10], m[11])
    {
    }
    void get(float m[12]) const
    {
        const float v[12] = {x00, x10, x20, x30, x01, x11, x21, x31, x02, x12, x22, x32};
        for (int i = 0; i < 12; i++) m[i] = v[i];
    }
    static Matrix identity() { return Matrix(); }
    static Matrix rotate(const Vector3D axis, const double angle)
    {
        const float a[3] = {axis.x, axis.y, axis.z};
        float m[12];
        pt_matrix_rotate(a, angle, m);
        return Matrix(m);
    }
    static Matrix rotateX(double angle) { return rotate(Vector3D(1, 0, 0), angle); }
    static Matrix rotateY(double angle) { return rotate(Vector3D(0, 1, 0), angle); }
    static Matrix rotateZ(double angle) { return rotate(Vector3D(0, 0, 1), angle); }
    static Matrix translate(Vector3D p) { return translate(p.x, p.y, p.z); }
    static Matrix translate(float x, float y, float z) { return Matrix(1, 0, 0, x, 0, 1, 0, y, 0, 0, 1, z); }
    static Matrix scale(float x, float y, float z) { return Matrix(x, 0, 0, 0, 0, y, 0, 0, 0, 0, z, 0); }
    static Matrix scale(Vector3D s) { return scale(s.x, s.y, s.z); }
    static Matrix scale(float s) { return scale(s, s, s); }
    friend Matrix invert(const Matrix &m)
    {
        float a[12], o[12];
        m.get(a);
        ptCheck(pt_matrix_inverse(a, o)); /* std::domain_error if singular, transform.h:353-354 */
        return Matrix(o);
    }
    Matrix concat(Matrix rt) const
    {
        float a[12], b[12], o[12];
        get(a);
        rt.get(b);
        pt_matrix_concat(a, b, o);
        return Matrix(o);
    }
    Vector3D apply(Vector3D v) const
    {
        return Vector3D(v.x * x00 + v.y * x10 + v.z * x20 + x30, v.x * x01 + v.y * x11 + v.z * x21 + x31,
                        v.x * x02 + v.y * x12 + v.z * x22 + x32);
    }
};

/* ---------------------------------------------------------------- images -- */
/* Refcounted, immutable RGBA f32 image, row 0 on top (include/image.h:48-101). */
class Image
{
public:
    Image() {}
    /* src/image.cpp:49-83: format from the extension unless given; "png" or
     * "hdr"/"pic" */
    explicit Image(std::string fileName, std::string format = "")
    {
        if (format.empty()) {
            size_t dot = fileName.find_last_of('.');
            if (dot == std::string::npos)
                throw ImageLoadError("can't determine format");
            format = fileName.substr(dot + 1);
        }
        for (auto &c : format) c = (char)tolower((unsigned char)c);
        int (*rd)(const char *, float *, int *, int *);
        if (format == "png")
            rd = pt_png_read;
        else if (format == "hdr" || format == "pic")
            rd = pt_hdr_read;
        else
            throw ImageLoadError("invalid format"); /* src/image.cpp:327 */
        int w = 0, h = 0;
        if (rd(fileName.c_str(), nullptr, &w, &h) != PT_OK)
            throw ImageLoadError(pt_last_error());
        std::shared_ptr<std::vector<float>> px(new std::vector<float>((size_t)w * h * 4));
        if (rd(fileName.c_str(), px->data(), &w, &h) != PT_OK)
            throw ImageLoadError(pt_last_error());
        data_ = px, w_ = (unsigned)w, h_ = (unsigned)h;
    }
    Image(std::vector<float> rgba, unsigned w, unsigned h)
        : data_(new std::vector<float>(std::move(rgba))), w_(w), h_(h)
    {
        if (data_->size() != (size_t)w * h * 4)
            throw std::invalid_argument("Image: rgba size != w*h*4");
    }
    unsigned width() const { return w_; }
    unsigned height() const { return h_; }
    explicit operator bool() const { return data_ != nullptr; }
    bool operator!() const { return data_ == nullptr; }
    friend bool operator==(const Image &l, const Image &r) { return l.data_ == r.data_; }
    friend bool operator!=(const Image &l, const Image &r) { return l.data_ != r.data_; }
    Color getPixel(int x, int y) const /* src/image.cpp:366-380 */
    {
        if (!data_ || x < 0 || y < 0 || (unsigned)x >= w_ || (unsigned)y >= h_)
            return Color(0);
        const float *p = data_->data() + ((size_t)y * w_ + x) * 4;
        return Color(p[0], p[1], p[2]);
    }
    float getPixelAlpha(int x, int y) const
    {
        if (!data_ || x < 0 || y < 0 || (unsigned)x >= w_ || (unsigned)y >= h_)
            return 0;
        return (*data_)[((size_t)y * w_ + x) * 4 + 3];
    }
    const float *rgba() const { return data_ ? data_->data() : nullptr; }

private:
    std::shared_ptr<const std::vector<float>> data_;
    unsigned w_ = 0, h_ = 0;
};

class MutableImage /* include/image.h:103-212 */
{
public:
    MutableImage(unsigned w, unsigned h) : data_((size_t)w * h * 4, 0.0f), w_(w), h_(h) {}
    explicit MutableImage(const Image &img) : w_(img.width()), h_(img.height())
    {
        if (!img)
            throw std::runtime_error("can't create MutableImage from empty Image");
        data_.assign(img.rgba(), img.rgba() + (size_t)w_ * h_ * 4);
    }
    unsigned width() const { return w_; }
    unsigned height() const { return h_; }
    void setPixel(int x, int y, Color c)
    {
        if (x < 0 || y < 0 || (unsigned)x >= w_ || (unsigned)y >= h_)
            return;
        float *p = &data_[((size_t)y * w_ + x) * 4];
        p[0] = c.x, p[1] = c.y, p[2] = c.z;
    }
    Color getPixel(int x, int y) const
    {
        if (x < 0 || y < 0 || (unsigned)x >= w_ || (unsigned)y >= h_)
            return Color(0);
        const float *p = &data_[((size_t)y * w_ + x) * 4];
        return Color(p[0], p[1], p[2]);
    }
    void writeHDR(std::string fileName) const /* src/image.cpp:398-481 */
    {
        std::vector<float> rgb((size_t)w_ * h_ * 3);
        for (size_t i = 0; i < (size_t)w_ * h_; i++)
            for (int c = 0; c < 3; c++) rgb[3 * i + c] = data_[4 * i + c];
        if (pt_write_hdr(fileName.c_str(), rgb.data(), (int)w_, (int)h_) != PT_OK)
            throw ImageStoreError(pt_last_error());
    }
    operator Image() const { return Image(data_, w_, h_); }

private:
    std::vector<float> data_;
    unsigned w_, h_;
};

/* ------------------------------------------------------------------- Ray -- */
struct Ray /* include/ray.h:9-23 */
{
    Vector3D origin;
    Vector3D dir;
    Ray(Vector3D origin, Vector3D dir) : origin(origin), dir(dir) {}
    Vector3D getPoint(float t) const { return origin + t * dir; }
};

/* ------------------------------------------------------------- flattening -- */
class Texture;
struct Material;
class Object;

/* Builds one pt_scene from a reference-style object graph.  Shared materials,
 * textures and images are flattened once. */
class Flattener
{
public:
    explicit Flattener(pt_scene *s) : s(s) {}
    pt_scene *const s;
    inline pt_id texture(const Texture *t);
    inline pt_id material(const Material *m);
    pt_id image(const Image &im)
    {
        if (!im)
            throw std::invalid_argument("empty Image in a texture");
        auto it = images_.find(im.rgba());
        if (it != images_.end())
            return it->second;
        return images_[im.rgba()] = ptCheck(pt_image_from_rgba32f(s, im.rgba(), (int)im.width(), (int)im.height()));
    }

private:
    std::map<const void *, pt_id> textures_, materials_, images_;

public:
    /* the Material a flattened material id stands for (span queries) */
    const Material *material_of(pt_id id) const
    {
        for (const auto &kv : materials_)
            if (kv.second == id)
                return static_cast<const Material *>(kv.first);
        return nullptr;
    }
};

/* A private pt_scene holding one flattened object or texture: what the
 * query virtuals evaluate on the device. */
struct DeviceQueryScene
{
    pt_scene *s;
    Flattener f;
    pt_id id = -1;
    DeviceQueryScene() : s(pt_scene_create()), f(s)
    {
        if (!s)
            throw DeviceError(PT_ERR_DEVICE, pt_last_error());
    }
    ~DeviceQueryScene() { pt_scene_destroy(s); }
    DeviceQueryScene(const DeviceQueryScene &) = delete;
    DeviceQueryScene &operator=(const DeviceQueryScene &) = delete;
};

/* --------------------------------------------------------------- textures -- */
class Texture /* include/texture.h:10-27 */
{
public:
    virtual ~Texture() {}
    /* getColor / getFloat (texture.h:13-18).  The built-in classes answer on
     * the device (pt_tex_eval of this texture, flattened once); a user-defined
     * subclass overrides getColor as in the reference -- it then works on the
     * host -- and gets a device form (renders, device lookups) by giving its
     * body as device source (deviceGetColor below).
     * The built-in classes are final and their fields const (Image is
     * immutable too), so the flattened form cached on first use never goes
     * stale and no override can be bypassed by the device path. */
    virtual Color getColor(Vector3D pos) const
    {
        Color c;
        float v;
        eval(&pos, 1, &c, &v);
        return c;
    }
    virtual float getFloat(Vector3D pos) const
    {
        if (!device_form_ && !deviceGetFloat()) { /* the reference's default: the mean of getColor */
            Color c = getColor(pos);
            return (c.x + c.y + c.z) * (1.0f / 3.0f);
        }
        Color c;
        float v;
        eval(&pos, 1, &c, &v);
        return v;
    }
    /* many lookups in one device call: colors[i], values[i] at pos[i] */
    void getColors(const Vector3D *pos, size_t n, Color *colors, float *values) const { eval(pos, n, colors, values); }
    virtual Texture *duplicate() const = 0;
    virtual Texture *transform(const Matrix &) const { return nullptr; }
    /* The device form of a user-defined subclass (pt_tex_device): its getColor
     * -- and getFloat, if it overrides the default -- as device source over
     * `V3 p` and its parameters `const float *prm` (deviceParams).  Give the
     * same arithmetic as the host override and the device computes the same
     * bits (the module is built without FMA contraction). */
    virtual const char *deviceGetColor() const { return nullptr; }
    virtual const char *deviceGetFloat() const { return nullptr; }
    virtual std::vector<float> deviceParams() const { return std::vector<float>(); }
    virtual pt_id flatten(Flattener &f) const
    {
        const char *body = deviceGetColor();
        if (!body)
            throw DeviceError(PT_ERR_ARG, "a user-defined Texture subclass has no device form "
                                          "(override deviceGetColor)");
        const std::vector<float> prm = deviceParams();
        return ptCheck(pt_tex_device(f.s, body, deviceGetFloat(), prm.data(), (int)prm.size()));
    }

protected:
    Texture() = default;
    explicit Texture(bool device_form) : device_form_(device_form) {}

private:
    bool device_form_ = false;
    mutable std::shared_ptr<DeviceQueryScene> q_;
    void eval(const Vector3D *pos, size_t n, Color *colors, float *values) const
    {
        static_assert(sizeof(Vector3D) == 3 * sizeof(float), "Vector3D must be 3 packed floats");
        if (!q_) {
            std::shared_ptr<DeviceQueryScene> q(new DeviceQueryScene);
            q->id = flatten(q->f);
            q_ = q;
        }
        ptCheck(pt_tex_eval(q_->s, q_->id, reinterpret_cast<const float *>(pos), (int64_t)n,
                            reinterpret_cast<float *>(colors), values, 0));
    }
};

class ColorTexture final : public Texture /* texture.h:29-58 */
{
public:
    const Color color;
    ColorTexture(Color color) : Texture(true), color(color) {}
    ColorTexture(float r, float g, float b) : Texture(true), color(r, g, b) {}
    ColorTexture(float v) : Texture(true), color(v) {}
    Texture *duplicate() const override { return new ColorTexture(color); }
    Texture *transform(const Matrix &) const override { return new ColorTexture(color); }
    pt_id flatten(Flattener &f) const override { return ptCheck(pt_tex_color(f.s, color.x, color.y, color.z)); }
};

class TransformedTexture final : public Texture /* texture.h:60-90 */
{
public:
    TransformedTexture(const Matrix &m, Texture *t) : Texture(true), m(m), t(t) {}
    ~TransformedTexture() override { delete t; }
    Texture *duplicate() const override { return new TransformedTexture(m, t->duplicate()); }
    Texture *transform(const Matrix &m2) const override { return new TransformedTexture(m.concat(m2), t->duplicate()); }
    pt_id flatten(Flattener &f) const override
    {
        float a[12];
        m.get(a);
        return ptCheck(pt_tex_transformed(f.s, a, f.texture(t)));
    }

private:
    Matrix m;
    Texture *t;
};

inline Texture *transform(const Matrix &m, Texture *t) /* texture.h:92-98 */
{
    Texture *r = t->transform(m);
    return r ? r : new TransformedTexture(m, t->duplicate());
}

class ImageTexture final : public Texture /* image_texture.h:9-33 */
{
public:
    explicit ImageTexture(Image image) : Texture(true), image(image) {}
    Texture *duplicate() const override { return new ImageTexture(image); }
    pt_id flatten(Flattener &f) const override { return ptCheck(pt_tex_image(f.s, f.image(image))); }
    const Image image;
};

class ImageAlphaTexture final : public Texture /* image_texture.h:35-70 */
{
public:
    explicit ImageAlphaTexture(Image image) : Texture(true), image(image) {}
    Texture *duplicate() const override { return new ImageAlphaTexture(image); }
    pt_id flatten(Flattener &f) const override { return ptCheck(pt_tex_image_alpha(f.s, f.image(image))); }
    const Image image;
};

class ImageSkyboxTexture final : public Texture /* image_texture.h:72-115 */
{
public:
    ImageSkyboxTexture(Image top, Image bottom, Image left, Image right, Image front, Image back)
        : Texture(true), faces{top, bottom, left, right, front, back}
    {
    }
    Texture *duplicate() const override
    {
        return new ImageSkyboxTexture(faces[0], faces[1], faces[2], faces[3], faces[4], faces[5]);
    }
    pt_id flatten(Flattener &f) const override
    {
        pt_id id[6];
        for (int i = 0; i < 6; i++) id[i] = f.image(faces[i]);
        return ptCheck(pt_tex_skybox(f.s, id[0], id[1], id[2], id[3], id[4], id[5]));
    }
    const Image faces[6];
};

class ImageSkyboxAlphaTexture final : public Texture /* image_texture.h:117-181 */
{
public:
    ImageSkyboxAlphaTexture(Image top, Image bottom, Image left, Image right, Image front, Image back)
        : Texture(true), faces{top, bottom, left, right, front, back}
    {
    }
    Texture *duplicate() const override
    {
        return new ImageSkyboxAlphaTexture(faces[0], faces[1], faces[2], faces[3], faces[4], faces[5]);
    }
    pt_id flatten(Flattener &f) const override
    {
        pt_id id[6];
        for (int i = 0; i < 6; i++) id[i] = f.image(faces[i]);
        return ptCheck(pt_tex_skybox_alpha(f.s, id[0], id[1], id[2], id[3], id[4], id[5]));
    }
    const Image faces[6];
};

/* owning single-child wrappers: FilterTexture (filter_texture.h:8-28) and
 * TransformTexture (transform_texture.h:8-31) */
class WrapTexture : public Texture
{
public:
    explicit WrapTexture(Texture *t) : Texture(true), t(t) {}
    ~WrapTexture() override { delete t; }

protected:
    Texture *const t;
};

class MultiplyTexture final : public WrapTexture /* filter_texture.h:30-48 */
{
public:
    MultiplyTexture(Color factor, Texture *t) : WrapTexture(t), factor(factor) {}
    Texture *duplicate() const override { return new MultiplyTexture(factor, t->duplicate()); }
    pt_id flatten(Flattener &f) const override
    {
        return ptCheck(pt_tex_multiply(f.s, factor.x, factor.y, factor.z, f.texture(t)));
    }
    const Color factor;
};

class LogTexture final : public WrapTexture /* filter_texture.h:50-80 */
{
public:
    explicit LogTexture(Texture *t) : WrapTexture(t) {}
    Texture *duplicate() const override { return new LogTexture(t->duplicate()); }
    pt_id flatten(Flattener &f) const override { return ptCheck(pt_tex_log(f.s, f.texture(t))); }
};

class MirrorBallSkymapTexture final : public WrapTexture /* transform_texture.h:33-59 */
{
public:
    explicit MirrorBallSkymapTexture(Texture *t) : WrapTexture(t) {}
    Texture *duplicate() const override { return new MirrorBallSkymapTexture(t->duplicate()); }
    pt_id flatten(Flattener &f) const override { return ptCheck(pt_tex_mirrorball(f.s, f.texture(t))); }
};

class SphericalCoordinatesSkymapTexture final : public WrapTexture /* :61-85 */
{
public:
    explicit SphericalCoordinatesSkymapTexture(Texture *t) : WrapTexture(t) {}
    Texture *duplicate() const override { return new SphericalCoordinatesSkymapTexture(t->duplicate()); }
    pt_id flatten(Flattener &f) const override { return ptCheck(pt_tex_spherical(f.s, f.texture(t))); }
};

/* --------------------------------------------------------------- material -- */
struct Material /* include/material.h:10-37 */
{
    Texture *reflect;
    Texture *scatter_coefficient;
    Texture *emissive;
    Texture *transmit;
    float ior;
    Texture *transmit_reflect_coefficient;
    Material(Texture *reflect = new ColorTexture(1), Texture *scatter_coefficient = new ColorTexture(1),
             Texture *emissive = new ColorTexture(0), Texture *transmit = new ColorTexture(0), float ior = 1,
             Texture *transmit_reflect_coefficient = new ColorTexture(0))
        : reflect(reflect), scatter_coefficient(scatter_coefficient), emissive(emissive), transmit(transmit),
          ior(ior), transmit_reflect_coefficient(transmit_reflect_coefficient)
    {
    }
    ~Material()
    {
        delete reflect;
        delete scatter_coefficient;
        delete emissive;
        delete transmit;
        delete transmit_reflect_coefficient;
    }
    Material *duplicate() const
    {
        return new Material(reflect->duplicate(), scatter_coefficient->duplicate(), emissive->duplicate(),
                            transmit->duplicate(), ior, transmit_reflect_coefficient->duplicate());
    }
    Material(const Material &) = delete;
    Material &operator=(const Material &) = delete;
};

inline Material *transform(const Matrix &m, const Material *mat) /* material.h:39-43 */
{
    return new Material(transform(m, mat->reflect), transform(m, mat->scatter_coefficient),
                        transform(m, mat->emissive), transform(m, mat->transmit), mat->ior,
                        transform(m, mat->transmit_reflect_coefficient));
}

inline pt_id Flattener::texture(const Texture *t)
{
    auto it = textures_.find(t);
    if (it != textures_.end())
        return it->second;
    pt_id id = t->flatten(*this);
    return textures_[t] = id;
}

inline pt_id Flattener::material(const Material *m)
{
    if (!m)
        throw std::invalid_argument("null material"); /* path-trace.h:77 asserts it */
    auto it = materials_.find(m);
    if (it != materials_.end())
        return it->second;
    pt_id id = ptCheck(pt_material(s, texture(m->reflect), texture(m->scatter_coefficient), texture(m->emissive),
                                   texture(m->transmit), m->ior, texture(m->transmit_reflect_coefficient)));
    return materials_[m] = id;
}

/* ------------------------------------------------------------------- spans -- */
class Span /* include/span.h:12-120 */
{
public:
    float start = 0;
    Vector3D startNormal;
    const Material *startMaterial = nullptr;
    float end = 0;
    Vector3D endNormal;
    const Material *endMaterial = nullptr;
    Span() = default;
    Span(float start, Vector3D startNormal, const Material *startMaterial, float end, Vector3D endNormal,
         const Material *endMaterial)
        : start(start), startNormal(startNormal), startMaterial(startMaterial), end(end), endNormal(endNormal),
          endMaterial(endMaterial)
    {
    }
    virtual ~Span() {}
    bool isEmpty() const { return end <= start; }
    explicit operator bool() const { return end > start; }
    bool operator!() const { return end <= start; }
};

class SpanIterator /* include/span.h:129-171 */
{
public:
    virtual const Span &operator*() const = 0;
    virtual const Span *operator->() const = 0;
    virtual bool isAtEnd() const = 0;
    virtual void next() = 0;
    virtual void init(const Ray &ray) = 0;
    virtual ~SpanIterator() {}
    bool operator!() const { return isAtEnd(); }
    explicit operator bool() const { return !isAtEnd(); }
    void operator++(int) { next(); }
    const SpanIterator &operator++()
    {
        next();
        return *this;
    }

protected:
    SpanIterator() = default;
    SpanIterator(const SpanIterator &) = delete;
    SpanIterator &operator=(const SpanIterator &) = delete;
};

/* ----------------------------------------------------------------- objects -- */
class Object /* include/object.h:10-24 */
{
public:
    virtual ~Object() {}
    /* object.h:14: the object's span iterator.  Built-in objects answer on the
     * device: init(ray) runs pt_query_spans on this object's flattened copy and
     * next() walks the returned list (bit-identical to the reference's lazy
     * iterators, Difference quirk included).  A user-defined subclass
     * overrides it as in the reference (host-side), and gets a device form --
     * renders, device span queries -- when its iterator yields one span per
     * ray and it returns that span's arithmetic as device source
     * (deviceSpan / deviceNormal below, pt_object_device). */
    inline virtual SpanIterator *makeSpanIterator() const;
    virtual Object *transform(const Matrix &) const { return nullptr; }
    virtual Object *duplicate() const = 0;
    /* The device form of a user-defined subclass: the bodies of
     * bool span(V3 o, V3 d, float &t0, float &t1) and V3 normal(V3 p) over
     * its parameters `const float *prm` (deviceParams), and its material. */
    virtual const char *deviceSpan() const { return nullptr; }
    virtual const char *deviceNormal() const { return nullptr; }
    virtual std::vector<float> deviceParams() const { return std::vector<float>(); }
    virtual const Material *deviceMaterial() const { return nullptr; }
    inline virtual pt_id flatten(Flattener &f) const;
};

inline pt_id Object::flatten(Flattener &f) const
{
    const char *sp = deviceSpan(), *nb = deviceNormal();
    if (!sp || !nb || !deviceMaterial())
        throw DeviceError(PT_ERR_ARG, "a user-defined Object subclass has no device form "
                                      "(override deviceSpan, deviceNormal and deviceMaterial)");
    const std::vector<float> prm = deviceParams();
    return ptCheck(pt_object_device(f.s, sp, nb, prm.data(), (int)prm.size(), f.material(deviceMaterial())));
}


/* The device-served SpanIterator of a built-in object (one query per init). */
class DeviceSpanIterator : public SpanIterator
{
public:
    explicit DeviceSpanIterator(const Object *o) : q_(new DeviceQueryScene)
    {
        q_->id = o->flatten(q_->f);
    }
    /* tracePixel's device side: this iterator's object as a render root
     * (set once), npixels pixel indices of a grid grid_width wide */
    void renderPixels(const int32_t *pixels, int64_t npixels, int W, int H, int grid_width, int spp, int depth,
                      float sw, float sh, float dist, uint64_t seed, int order, float *rgb) const
    {
        if (!root_set_) {
            ptCheck(pt_set_root(q_->s, q_->id));
            root_set_ = true;
        }
        pt_render_params p = {};
        p.width = W, p.height = H, p.spp = spp, p.depth = depth;
        p.screen_w = sw, p.screen_h = sh, p.screen_dist = dist;
        p.seed = seed, p.order = order, p.grid_width = grid_width;
        p.pixels = pixels, p.npixels = npixels;
        ptCheck(pt_render(q_->s, &p, rgb, nullptr));
    }
    /* traceRay's device side: n rays of 7 floats (origin, direction, strength),
     * spp samples each, engine keys ray_begin + k (pt_trace_rays) */
    void renderRays(const float *rays, int64_t n, int spp, int depth, uint64_t seed, int order, int64_t ray_begin,
                    float *rgb) const
    {
        if (!root_set_) {
            ptCheck(pt_set_root(q_->s, q_->id));
            root_set_ = true;
        }
        pt_trace_params p = {};
        p.spp = spp, p.depth = depth, p.seed = seed, p.order = order, p.ray_begin = ray_begin;
        ptCheck(pt_trace_rays(q_->s, &p, rays, n, rgb, nullptr));
    }
    const Span &operator*() const override { return spans_.at(k_); }
    const Span *operator->() const override { return &spans_.at(k_); }
    bool isAtEnd() const override { return k_ >= spans_.size(); }
    void next() override
    {
        if (k_ < spans_.size())
            k_++;
    }
    void init(const Ray &ray) override
    {
        const float r[6] = {ray.origin.x, ray.origin.y, ray.origin.z, ray.dir.x, ray.dir.y, ray.dir.z};
        int32_t count = 0;
        std::vector<pt_span> buf(8);
        ptCheck(pt_query_spans(q_->s, q_->id, r, 1, (int)buf.size(), buf.data(), &count, 0));
        if (count > (int32_t)buf.size()) {
            buf.resize((size_t)count);
            ptCheck(pt_query_spans(q_->s, q_->id, r, 1, count, buf.data(), &count, 0));
        }
        spans_.clear();
        for (int32_t i = 0; i < count; i++) {
            const pt_span &p = buf[(size_t)i];
            spans_.push_back(Span(p.t_start, Vector3D(p.n_start[0], p.n_start[1], p.n_start[2]),
                                  q_->f.material_of(p.mat_start), p.t_end,
                                  Vector3D(p.n_end[0], p.n_end[1], p.n_end[2]), q_->f.material_of(p.mat_end)));
        }
        k_ = 0;
    }

private:
    std::unique_ptr<DeviceQueryScene> q_;
    std::vector<Span> spans_;
    size_t k_ = 0;
    mutable bool root_set_ = false;
};

inline SpanIterator *Object::makeSpanIterator() const { return new DeviceSpanIterator(this); }

/* -------------------------------------------------------------- tracePixel -- */
const int DefaultRayDepth = 16;          /* include/path-trace.h:57  */
const int DefaultSampleCount = 200;      /* include/path-trace.h:167 */
const float DefaultScreenWidth = 4.0 / 3.0, DefaultScreenHeight = 1.0, DefaultScreenDistance = 2.0; /* :168-170 */

/* The engine argument of tracePixel (include/path-trace.h:187-201 takes the
 * caller's `T &randomEngine` and draws every sample of every pixel from it in
 * sequence).  The device gives each (pixel, sample) an engine of its own,
 * keyed from a run seed (include/pt/pt_engine.h), so the samples of many
 * pixels run side by side: calls with the same FrameEngine return, pixel by
 * pixel, the bits Renderer::render returns for the frame with that seed and
 * order -- in any call order, from any thread. */
struct FrameEngine
{
    uint64_t seed;
    int order;
    /* traceRay / float-coordinate tracePixel calls key their samples by a ray
     * index: the next one this engine hands out (successive calls draw fresh
     * streams, as successive calls of the reference draw on from its engine;
     * not thread-safe, like the reference's engines) */
    uint64_t rays = 0;
    explicit FrameEngine(uint64_t seed = 0x5EED, int order = PT_ORDER_FAST) : seed(seed), order(order) {}
};

/* the global engine of the non-template overload (the reference's defaultRandomEngine, path-trace.h:56) */
inline FrameEngine &defaultFrameEngine()
{
    static FrameEngine e;
    return e;
}

/* tracePixel(SpanIterator &, int px, int py, ...) of include/path-trace.h:187-201
 * over a batch: colors[k] = the mean radiance of pixel (px[k], py[k]).  The span
 * iterator must be a built-in object's (Object::makeSpanIterator): its object is
 * the scene the device renders.  One device launch for the in-frame pixels.
 * A pixel's engine keys depend on the pixel alone, never on the rest of the
 * batch: pixels with x < screenXResolution are keyed on the frame's grid (the
 * bits Renderer::render returns); pixels past the right edge (the adaptive
 * caller's block corners at x == screenXResolution, src/test.cpp:466-499) are
 * rendered per column x in a launch of their own, keyed on a grid x + 1 wide
 * with a run seed derived from (engine.seed, x), so they can share no sample
 * stream with an in-frame pixel. */
inline uint64_t edgeColumnSeed(uint64_t seed, int x)
{
    uint64_t z = seed ^ (0xD1B54A32D192ED03ull * (uint64_t)(uint32_t)(x + 1));
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

/* the engine key of pixel (px, py) on a frame W wide (a column past the right
 * edge is keyed on its own grid, x + 1 wide); throws on a coordinate no key exists for */
inline int64_t pixelKeyIndex(int px, int py, int W)
{
    if (px < 0 || py < 0)
        throw std::invalid_argument("tracePixel: negative pixel coordinate");
    const int gw = px < W ? W : px + 1;
    const int64_t i = (int64_t)py * gw + px;
    if (i > INT32_MAX)
        throw std::invalid_argument("tracePixel: pixel index out of range");
    return i;
}

inline void tracePixels(SpanIterator &spanIterator, const int32_t *px, const int32_t *py, size_t n, Color *colors,
                        int screenXResolution, int screenYResolution, int sampleCount, int rayDepth, float screenWidth,
                        float screenHeight, float screenDistance, const FrameEngine &engine)
{
    DeviceSpanIterator *it = dynamic_cast<DeviceSpanIterator *>(&spanIterator);
    if (!it)
        throw DeviceError(PT_ERR_ARG, "tracePixel: needs the span iterator of a built-in object "
                                      "(Object::makeSpanIterator)");
    if (n == 0)
        return;
    static_assert(sizeof(Color) == 3 * sizeof(float), "Color must be 3 packed floats");
    const int W = screenXResolution;
    std::vector<int32_t> in_pix;
    std::vector<size_t> in_at;
    std::map<int, std::vector<size_t>> edge; /* column x >= W -> batch positions */
    for (size_t k = 0; k < n; k++) {
        const int64_t i = pixelKeyIndex(px[k], py[k], W);
        if (px[k] < W) {
            in_pix.push_back((int32_t)i);
            in_at.push_back(k);
        } else {
            edge[px[k]].push_back(k);
        }
    }
    std::vector<float> rgb;
    auto launch = [&](const std::vector<int32_t> &pix, const std::vector<size_t> &at, int gw, uint64_t seed) {
        rgb.assign(3 * pix.size(), 0.0f);
        it->renderPixels(pix.data(), (int64_t)pix.size(), W, screenYResolution, gw, sampleCount, rayDepth,
                         screenWidth, screenHeight, screenDistance, seed, engine.order, rgb.data());
        for (size_t j = 0; j < at.size(); j++)
            colors[at[j]] = Color(rgb[3 * j], rgb[3 * j + 1], rgb[3 * j + 2]);
    };
    if (!in_pix.empty())
        launch(in_pix, in_at, W, engine.seed);
    for (const auto &col : edge) {
        std::vector<int32_t> pix;
        for (size_t k : col.second)
            pix.push_back((int32_t)((int64_t)py[k] * (col.first + 1) + col.first));
        launch(pix, col.second, col.first + 1, edgeColumnSeed(engine.seed, col.first));
    }
}

inline Color tracePixel(SpanIterator &spanIterator, int px, int py, int screenXResolution, int screenYResolution,
                        int sampleCount, int rayDepth, float screenWidth, float screenHeight, float screenDistance,
                        FrameEngine &randomEngine)
{
    const int32_t x = px, y = py;
    Color c;
    tracePixels(spanIterator, &x, &y, 1, &c, screenXResolution, screenYResolution, sampleCount, rayDepth,
                screenWidth, screenHeight, screenDistance, randomEngine);
    return c;
}

/* Any other engine type T (unsigned operator()(), as include/vector3d.h:14-34
 * requires of it -- e.g. the reference's DefaultRandomEngine): two of its
 * draws make the run seed of this call, so successive calls see fresh
 * streams as with the reference's shared engine. */
template <typename T>
inline Color tracePixel(SpanIterator &spanIterator, int px, int py, int screenXResolution, int screenYResolution,
                        int sampleCount, int rayDepth, float screenWidth, float screenHeight, float screenDistance,
                        T &randomEngine)
{
    const uint64_t hi = (uint32_t)randomEngine(), lo = (uint32_t)randomEngine();
    FrameEngine e((hi << 32) | lo);
    return tracePixel(spanIterator, px, py, screenXResolution, screenYResolution, sampleCount, rayDepth,
                      screenWidth, screenHeight, screenDistance, e);
}

/* the non-template overload (include/path-trace.h:203-206): the global engine */
inline Color tracePixel(SpanIterator &spanIterator, int px, int py, int screenXResolution, int screenYResolution,
                        int sampleCount = DefaultSampleCount, int rayDepth = DefaultRayDepth,
                        float screenWidth = DefaultScreenWidth, float screenHeight = DefaultScreenHeight,
                        float screenDistance = DefaultScreenDistance)
{
    return tracePixel(spanIterator, px, py, screenXResolution, screenYResolution, sampleCount, rayDepth, screenWidth,
                      screenHeight, screenDistance, defaultFrameEngine());
}

static inline DeviceSpanIterator &deviceIterator(SpanIterator &spanIterator, const char *who)
{
    DeviceSpanIterator *it = dynamic_cast<DeviceSpanIterator *>(&spanIterator);
    if (!it)
        throw DeviceError(PT_ERR_ARG, std::string(who) + ": needs the span iterator of a built-in object "
                                                          "(Object::makeSpanIterator)");
    return *it;
}

/* traceRay<T>(ray, spanIterator, depth, engine, strength) of include/path-
 * trace.h:58-165 over a batch, in one device launch: colors[k] = the mean of
 * `samples` traceRay values of rays[k] with strengths[k] (nullptr: 1), sample
 * s of ray k drawing from the engine keyed (engine.seed, engine.rays + k, s);
 * the engine then hands out the next n keys. */
inline void traceRays(SpanIterator &spanIterator, const Ray *rays, const float *strengths, size_t n, Color *colors,
                      int rayDepth, FrameEngine &engine, int samples = 1)
{
    DeviceSpanIterator &it = deviceIterator(spanIterator, "traceRay");
    if (n == 0)
        return;
    std::vector<float> r(7 * n);
    for (size_t k = 0; k < n; k++) {
        const float v[7] = {rays[k].origin.x, rays[k].origin.y, rays[k].origin.z, rays[k].dir.x,
                            rays[k].dir.y,    rays[k].dir.z,    strengths ? strengths[k] : 1.0f};
        std::copy(v, v + 7, &r[7 * k]);
    }
    static_assert(sizeof(Color) == 3 * sizeof(float), "Color must be 3 packed floats");
    it.renderRays(r.data(), (int64_t)n, samples, rayDepth, engine.seed, engine.order, (int64_t)engine.rays,
                  reinterpret_cast<float *>(colors));
    engine.rays += n;
}

/* traceRay with a FrameEngine: one ray, the engine's next key */
inline Color traceRay(const Ray &ray, SpanIterator &spanIterator, int depth, FrameEngine &randomEngine,
                      float strength = 1.0f)
{
    Color c;
    traceRays(spanIterator, &ray, &strength, 1, &c, depth, randomEngine);
    return c;
}

/* traceRay with any other engine type T (unsigned operator()(), include/
 * vector3d.h:14-34): two of its draws make the run seed of this call */
template <typename T>
inline Color traceRay(const Ray &ray, SpanIterator &spanIterator, int depth, T &randomEngine, float strength = 1.0f)
{
    const uint64_t hi = (uint32_t)randomEngine(), lo = (uint32_t)randomEngine();
    FrameEngine e((hi << 32) | lo);
    return traceRay(ray, spanIterator, depth, e, strength);
}

/* traceRay(ray, spanIterator[, depth]) with the global engine (path-trace.h:59's defaults) */
inline Color traceRay(const Ray &ray, SpanIterator &spanIterator, int depth = DefaultRayDepth)
{
    return traceRay(ray, spanIterator, depth, defaultFrameEngine(), 1.0f);
}

/* tracePixel's float-coordinate overload (include/path-trace.h:172-185): the
 * ray through (px, py) -- no jitter, computed in float as the reference does --
 * traced sampleCount times and averaged, in one device launch. */
inline Color tracePixel(SpanIterator &spanIterator, float px, float py, float screenXResolution,
                        float screenYResolution, int sampleCount, int rayDepth, float screenWidth, float screenHeight,
                        float screenDistance, FrameEngine &randomEngine)
{
    const float x = 2 * px / screenXResolution - 1;
    const float y = 1 - 2 * py / screenYResolution;
    const Ray ray(Vector3D(0, 0, 0), Vector3D(x * screenWidth, y * screenHeight, -screenDistance));
    const float strength = 1.0f;
    Color c;
    traceRays(spanIterator, &ray, &strength, 1, &c, rayDepth, randomEngine, sampleCount);
    return c;
}
template <typename T>
inline Color tracePixel(SpanIterator &spanIterator, float px, float py, float screenXResolution,
                        float screenYResolution, int sampleCount, int rayDepth, float screenWidth, float screenHeight,
                        float screenDistance, T &randomEngine)
{
    const uint64_t hi = (uint32_t)randomEngine(), lo = (uint32_t)randomEngine();
    FrameEngine e((hi << 32) | lo);
    return tracePixel(spanIterator, px, py, screenXResolution, screenYResolution, sampleCount, rayDepth, screenWidth,
                      screenHeight, screenDistance, e);
}

/* Coalesces the per-pixel tracePixel calls of many host threads into device
 * batches: the shape of the reference demo's RenderBlock pool, whose threads
 * each call tracePixel for one pixel at a time (src/test.cpp:441-465, the call
 * at :450; one thread per core, :204).  tracePixel() is thread-safe and blocks
 * until its pixel's batch is traced; a batch launches when maxBatch calls wait
 * or maxWaitUs after its first call.  Pixels keep the bits tracePixels gives
 * them alone (keys depend on the pixel only). */
class PixelBatcher
{
public:
    PixelBatcher(SpanIterator &spanIterator, int screenXResolution, int screenYResolution, int sampleCount,
                 int rayDepth, float screenWidth, float screenHeight, float screenDistance,
                 const FrameEngine &engine = FrameEngine(), size_t maxBatch = 4096, int maxWaitUs = 200)
        : it_(spanIterator), W_(screenXResolution), H_(screenYResolution), spp_(sampleCount), depth_(rayDepth),
          sw_(screenWidth), sh_(screenHeight), dist_(screenDistance), engine_(engine),
          maxBatch_(maxBatch ? maxBatch : 1), maxWaitUs_(maxWaitUs), worker_([this] { run(); })
    {
    }
    ~PixelBatcher()
    {
        {
            std::lock_guard<std::mutex> g(m_);
            stop_ = true;
        }
        cv_.notify_all();
        worker_.join();
    }
    PixelBatcher(const PixelBatcher &) = delete;
    PixelBatcher &operator=(const PixelBatcher &) = delete;

    Color tracePixel(int px, int py)
    {
        (void)pixelKeyIndex(px, py, W_); /* a bad coordinate fails its own caller, not the batch it would join */
        Req r;
        r.x = px, r.y = py;
        std::unique_lock<std::mutex> lk(m_);
        if (stop_)
            throw std::logic_error("PixelBatcher: stopped");
        queue_.push_back(&r);
        cv_.notify_all();
        done_.wait(lk, [&] { return r.done; });
        if (r.err)
            std::rethrow_exception(r.err);
        return r.c;
    }
    uint64_t launches() const
    {
        std::lock_guard<std::mutex> g(m_);
        return launches_;
    }
    uint64_t pixels() const
    {
        std::lock_guard<std::mutex> g(m_);
        return pixels_;
    }

private:
    struct Req
    {
        int x = 0, y = 0;
        Color c;
        bool done = false;
        std::exception_ptr err;
    };
    void run()
    {
        std::unique_lock<std::mutex> lk(m_);
        for (;;) {
            cv_.wait(lk, [&] { return stop_ || !queue_.empty(); });
            if (queue_.empty() && stop_)
                return;
            /* a batch launches at maxBatch, after maxWaitUs -- or as soon as
             * as many calls wait as the previous batch held: the steady state
             * of N threads each asking for one pixel at a time, which then
             * costs no batching window at all (a thread that stops calling
             * costs one window, after which the size adapts) */
            cv_.wait_for(lk, std::chrono::microseconds(maxWaitUs_), [&] {
                return stop_ || queue_.size() >= maxBatch_ || (lastBatch_ > 0 && queue_.size() >= lastBatch_);
            });
            const size_t n = std::min(queue_.size(), maxBatch_);
            lastBatch_ = n;
            std::vector<Req *> batch(queue_.begin(), queue_.begin() + (std::ptrdiff_t)n);
            queue_.erase(queue_.begin(), queue_.begin() + (std::ptrdiff_t)n);
            lk.unlock();
            std::vector<int32_t> xs(n), ys(n);
            std::vector<Color> cs(n);
            std::exception_ptr err;
            for (size_t k = 0; k < n; k++) xs[k] = batch[k]->x, ys[k] = batch[k]->y;
            try {
                tracePixels(it_, xs.data(), ys.data(), n, cs.data(), W_, H_, spp_, depth_, sw_, sh_, dist_, engine_);
            } catch (...) {
                err = std::current_exception();
            }
            lk.lock();
            for (size_t k = 0; k < n; k++) batch[k]->c = cs[k], batch[k]->err = err, batch[k]->done = true;
            launches_++;
            pixels_ += n;
            done_.notify_all();
        }
    }
    SpanIterator &it_;
    const int W_, H_, spp_, depth_;
    const float sw_, sh_, dist_;
    const FrameEngine engine_;
    const size_t maxBatch_;
    const int maxWaitUs_;
    mutable std::mutex m_;
    std::condition_variable cv_, done_;
    std::vector<Req *> queue_;
    size_t lastBatch_ = 0;
    bool stop_ = false;
    uint64_t launches_ = 0, pixels_ = 0;
    std::thread worker_; /* last: started once every member above is constructed */
};

class TransformedObject : public Object /* object.h:26-98 */
{
public:
    TransformedObject(const Matrix &m, Object *o) : m(m), o(o) {}
    ~TransformedObject() override { delete o; }
    Object *transform(const Matrix &m2) const override { return new TransformedObject(m.concat(m2), o->duplicate()); }
    Object *duplicate() const override { return new TransformedObject(m, o->duplicate()); }
    pt_id flatten(Flattener &f) const override
    {
        float a[12];
        m.get(a);
        return ptCheck(pt_transformed(f.s, a, o->flatten(f)));
    }

private:
    Matrix m;
    Object *o;
};

inline Object *transform(const Matrix &m, Object *o) /* object.h:100-106 */
{
    Object *r = o->transform(m);
    return r ? r : new TransformedObject(m, o->duplicate());
}

class Sphere : public Object /* include/sphere.h, src/sphere.cpp */
{
public:
    Sphere(Vector3D center, float r, const Material *material) : center(center), r(r), material(material) {}
    Object *duplicate() const override { return new Sphere(center, r, material); }
    pt_id flatten(Flattener &f) const override
    {
        return ptCheck(pt_sphere(f.s, center.x, center.y, center.z, r, f.material(material)));
    }

private:
    Vector3D center;
    float r;
    const Material *material;
};

class Plane : public Object /* include/plane.h, src/plane.cpp:6-14 */
{
public:
    Plane(Vector3D normal, float d, const Material *material) : normal(normal), d(d), material(material) {}
    Plane(Vector3D normal, Vector3D pos, const Material *material)
        : normal(normal), d(-dot(normal, pos)), material(material)
    {
    }
    Object *duplicate() const override { return new Plane(normal, d, material); }
    pt_id flatten(Flattener &f) const override
    {
        return ptCheck(pt_plane(f.s, normal.x, normal.y, normal.z, d, f.material(material)));
    }

private:
    Vector3D normal;
    float d;
    const Material *material;
};

template <class Self, int OP>
class CsgObject : public Object
{
public:
    CsgObject(Object *a, Object *b) : a(a), b(b) {}
    ~CsgObject() override
    {
        delete a;
        delete b;
    }
    Object *duplicate() const override { return new Self(a->duplicate(), b->duplicate()); }
    /* union.h:21, intersection.h:21, difference.h:21 transform `a` twice (the
     * second operand is dropped) -- kept so that transformed scenes match. */
    Object *transform(const Matrix &m) const override
    {
        return new Self(PathTrace::transform(m, a), PathTrace::transform(m, a));
    }
    pt_id flatten(Flattener &f) const override
    {
        pt_id ia = a->flatten(f);
        pt_id ib = b->flatten(f);
        return ptCheck(pt_csg(f.s, OP, ia, ib));
    }

private:
    Object *const a;
    Object *const b;
};

class Union : public CsgObject<Union, PT_CSG_UNION> /* include/union.h, src/union.cpp */
{
public:
    using CsgObject::CsgObject;
};
class Intersection : public CsgObject<Intersection, PT_CSG_INTERSECTION> /* src/intersection.cpp */
{
public:
    using CsgObject::CsgObject;
};
class Difference : public CsgObject<Difference, PT_CSG_DIFFERENCE> /* src/difference.cpp */
{
public:
    using CsgObject::CsgObject;
};

inline Object *unionArray(Object *array[], int start, int end) /* src/test.cpp:52-64 */
{
    if (end - start == 1)
        return array[start];
    if (end - start == 2)
        return new Union(array[start], array[start + 1]);
    int split = (end - start) / 2 + start;
    return new Union(unionArray(array, start, split), unionArray(array, split, end));
}

/* ---------------------------------------------------------------- renderer -- */
/* Replaces world->makeSpanIterator() + tracePixel<T> per pixel.  The object
 * graph is flattened once; the Renderer does not keep pointers into it. */
class Renderer
{
public:
    struct Settings
    {
        int width = 0, height = 0;  /* screenXResolution, screenYResolution       */
        int sampleCount = 1;        /* tracePixel sampleCount                       */
        int rayDepth = 16;          /* tracePixel/traceRay depth                    */
        float screenWidth = 0, screenHeight = 0, screenDistance = 0; /* 0 = the demo's
                                       convention: W, H, 2 min(W, H) (src/test.cpp:450) */
        uint64_t seed = 0x5EED;     /* run seed of the per-(pixel, sample) engine   */
        int order = PT_ORDER_FAST;
        int device = 0;
        int64_t maxBufferBytes = 0;
    };

    explicit Renderer(const Object *world) : s_(pt_scene_create())
    {
        if (!s_)
            throw DeviceError(PT_ERR_DEVICE, pt_last_error());
        try {
            Flattener f(s_);
            ptCheck(pt_set_root(s_, world->flatten(f)));
        } catch (...) {
            pt_scene_destroy(s_);
            throw;
        }
    }
    ~Renderer() { pt_scene_destroy(s_); }
    Renderer(const Renderer &) = delete;
    Renderer &operator=(const Renderer &) = delete;

    pt_scene *handle() const { return s_; }

    /* Mean radiance per pixel (tracePixel's return value), row-major, for the
     * whole frame -- or, with pixels != nullptr, for those pixel indices. */
    std::vector<Color> render(const Settings &st, const int32_t *pixels = nullptr, int64_t npixels = 0,
                              pt_render_stats *stats = nullptr) const
    {
        pt_render_params p = params(st, pixels, npixels);
        int64_t n = pixels ? npixels : (int64_t)st.width * st.height;
        std::vector<Color> out((size_t)n);
        static_assert(sizeof(Color) == 3 * sizeof(float), "Color must be 3 packed floats");
        ptCheck(pt_render(s_, &p, reinterpret_cast<float *>(out.data()), stats));
        return out;
    }

    /* Device-side variant: fb is a W*H*3 float device buffer, stream a hipStream_t. */
    void renderDevice(const Settings &st, float *fb, void *stream, const int32_t *pixels = nullptr,
                      int64_t npixels = 0, pt_render_stats *stats = nullptr) const
    {
        pt_render_params p = params(st, pixels, npixels);
        ptCheck(pt_render_device(s_, &p, fb, stream, stats));
    }

    /* The demo's adaptive image formation, RenderBlock::renderSquare
     * (src/test.cpp:423-507): 0 selects the demo's block size, interpolation
     * limit and colour threshold.  Returns the width*height image. */
    std::vector<Color> renderAdaptive(const Settings &st, int blockSize = 0, int maxInterp = 0, float minDelta = 0,
                                      pt_adaptive_params *info = nullptr, pt_render_stats *stats = nullptr) const
    {
        pt_render_params p = params(st, nullptr, 0);
        pt_adaptive_params ap = {};
        ap.block_size = blockSize, ap.max_interp = maxInterp, ap.min_delta = minDelta;
        std::vector<Color> out((size_t)st.width * st.height);
        ptCheck(pt_render_adaptive(s_, &p, &ap, reinterpret_cast<float *>(out.data()), stats));
        if (info)
            *info = ap;
        return out;
    }

    /* Compile / upload everything a render with these settings needs. */
    void prepare(const Settings &st) const
    {
        pt_render_params p = params(st, nullptr, 0);
        ptCheck(pt_prepare(s_, &p));
    }

    static pt_render_params params(const Settings &st, const int32_t *pixels, int64_t npixels)
    {
        pt_render_params p = {};
        p.width = st.width, p.height = st.height, p.spp = st.sampleCount, p.depth = st.rayDepth;
        const float dmin = (float)(st.width < st.height ? st.width : st.height);
        p.screen_w = st.screenWidth > 0 ? st.screenWidth : (float)st.width;
        p.screen_h = st.screenHeight > 0 ? st.screenHeight : (float)st.height;
        p.screen_dist = st.screenDistance > 0 ? st.screenDistance : 2 * dmin;
        p.seed = st.seed, p.order = st.order, p.device = st.device;
        p.pixels = pixels, p.npixels = npixels, p.max_buffer_bytes = st.maxBufferBytes;
        return p;
    }

private:
    pt_scene *s_;
};

/* SDL_SaveBMP of the demo's tone map (src/test.cpp:1037-1059). */
inline void writeBMP(const std::string &path, const std::vector<Color> &rgb, int w, int h, int count = 1)
{
    if (pt_write_bmp(path.c_str(), reinterpret_cast<const float *>(rgb.data()), w, h, count) != PT_OK)
        throw ImageStoreError(pt_last_error());
}

} // namespace PathTrace

#endif
