/*
 * oracle.cpp -- TEST INFRASTRUCTURE ONLY.  CPU restatement of the reference's
 * per-pixel Monte-Carlo path, used by tests/ as the parity checker, by
 * __graft_entry__.smoke() and by bench.py's cpu_baseline leg.  The product
 * (path-trace_amd/) never links, loads or calls anything in oracle/.
 *
 * Pinned against the reference itself: oracle/_ref/ptref runs the UNMODIFIED
 * reference sources and tests/golden/ freezes its outputs; tests check this
 * restatement against them bit-for-bit (tests/test_oracle_golden.py).
 *
 * Formulation differences from both the reference and the GPU kernel (kept on
 * purpose, so the three implementations cross-check each other):
 *   - span lists are evaluated EAGERLY (full sorted lists per CSG node) instead
 *     of the reference's lazy SpanIterator pull chain (include/span.h:129-171)
 *     or the GPU's lazy compact-span pull; the emitted sequence is identical
 *     because every node's next() is a pure function of its children's lists;
 *   - normals are computed eagerly, as the reference does (src/sphere.cpp:47-48),
 *     while the GPU recomputes them lazily for the chosen hit only.
 *
 * Two accumulation orders:
 *   ORDER_REFERENCE : retval += child, one child at a time (path-trace.h:162)
 *   ORDER_FAST      : the GPU fast path's order -- in a scatter loop with
 *                     scatter_coefficient > eps, a RUN is a maximal sequence of
 *                     consecutive LEAF children (depth-1 <= 0 or child strength
 *                     < eps, i.e. children that draw no random numbers).  The
 *                     run's terms w * child that are not exactly zero (some
 *                     channel != 0; NaN counts as non-zero) are dealt round-robin
 *                     to 64 lane sums: the k-th such term of the run is added to
 *                     lane k mod 64, each lane summing in order from +0.  Zero
 *                     terms change no lane sum (a lane sum that starts at +0 is
 *                     never -0), so where they fall does not matter.  At the run's
 *                     end retval += the pairwise tree of the 64 lane sums; a
 *                     non-leaf child closes the open run and is added on its own.
 *                     A pixel's samples are summed in blocks of 32 (pairwise
 *                     tree each, padded with -0.0f), blocks one after the
 *                     other (pixel_sum).
 */
#include "oracle_engine.h"
#include "scene_text.h"

#include <atomic>
#include <functional>
#include <cmath>
#include <cstring>
#include <fstream>
#include <map>
#include <memory>
#include <mutex>
#include <stdexcept>
#include <string>
#include <thread>
#include <vector>

namespace oracle
{

const float kEps = 1e-3f;          // include/misc.h:7
const float kMaxValue = 1e20f;     // include/misc.h:8

/* ---------------------------------------------------------------- math --- */
/* Vector3D semantics, include/vector3d.h:36-219.  Every operator keeps the
 * reference's evaluation order (dot = (x + y) + z of the products). */
struct V3
{
    float x, y, z;
    V3() : x(0), y(0), z(0) {}
    V3(float a, float b, float c) : x(a), y(b), z(c) {}
    explicit V3(float v) : x(v), y(v), z(v) {}
};
inline V3 operator+(V3 a, V3 b) { return V3(a.x + b.x, a.y + b.y, a.z + b.z); }
inline V3 operator-(V3 a, V3 b) { return V3(a.x - b.x, a.y - b.y, a.z - b.z); }
inline V3 operator*(V3 a, V3 b) { return V3(a.x * b.x, a.y * b.y, a.z * b.z); }
inline V3 operator*(V3 a, float s) { return V3(a.x * s, a.y * s, a.z * s); }
inline V3 operator*(float s, V3 a) { return V3(a.x * s, a.y * s, a.z * s); }
inline V3 operator/(V3 a, float s) { return V3(a.x / s, a.y / s, a.z / s); }
inline V3 operator-(V3 a) { return V3(-a.x, -a.y, -a.z); }
inline bool operator==(V3 a, V3 b) { return a.x == b.x && a.y == b.y && a.z == b.z; }
inline bool operator!=(V3 a, V3 b) { return a.x != b.x || a.y != b.y || a.z != b.z; }
inline float dot(V3 a, V3 b)
{
    V3 p = a * b;
    return p.x + p.y + p.z;
}
inline float length(V3 v) { return std::sqrt(dot(v, v)); } /* float sqrt, vector3d.h:111-114 */
inline V3 normalize(V3 v)
{
    float m = length(v);
    if (m == 0)
        m = 1;
    return v / m;
}

/* Vector3D::reflect, vector3d.h:186-190 */
inline V3 reflect(V3 d, V3 n)
{
    n = normalize(n);
    return d - (2 * dot(d, n)) * n;
}

inline bool bad_ior(float ior, V3 n, V3 d)
{
    return ior < kEps || ior > 1 / kEps || n == V3(0, 0, 0) || d == V3(0, 0, 0);
}

/* Vector3D::refractStrength, vector3d.h:191-202.  The final sqrt(sqrt(.)) is an
 * unqualified call inside namespace PathTrace with a float argument, which
 * resolves to ::sqrt(double): two double square roots, one rounding to float. */
inline float refract_strength(V3 d, float ior, V3 n)
{
    if (bad_ior(ior, n, d))
        return 0;
    n = normalize(n);
    V3 inc = normalize(d);
    float c = dot(inc, n);
    float r = 1 - ior * ior * (1 - c * c);
    if (r <= 0)
        return 0;
    return (float)::sqrt(::sqrt((double)r));
}

/* Vector3D::refract, vector3d.h:203-214 (float std::sqrt) */
inline V3 refract(V3 d, float ior, V3 n)
{
    if (bad_ior(ior, n, d))
        return V3(0, 0, 0);
    n = normalize(n);
    V3 inc = normalize(d);
    float c = dot(inc, n);
    float arg = 1 - ior * ior * (1 - c * c);
    if (arg < 0)
        return V3(0, 0, 0);
    return normalize(ior * inc - (ior * c + std::sqrt(arg)) * n);
}

/* Matrix (3x4 affine), include/transform.h:16-422; constructor order x00 x10 x20 x30 x01 ... */
struct M34
{
    float x00, x10, x20, x30, x01, x11, x21, x31, x02, x12, x22, x32;
    static M34 from(const float *f)
    {
        M34 m;
        memcpy(&m, f, sizeof(float) * 12);
        return m;
    }
    V3 apply(V3 v) const
    {
        return V3(v.x * x00 + v.y * x10 + v.z * x20 + x30, v.x * x01 + v.y * x11 + v.z * x21 + x31,
                  v.x * x02 + v.y * x12 + v.z * x22 + x32);
    }
    V3 apply_linear(V3 v) const
    {
        return V3(v.x * x00 + v.y * x10 + v.z * x20, v.x * x01 + v.y * x11 + v.z * x21,
                  v.x * x02 + v.y * x12 + v.z * x22);
    }
    /* transform.h:342-383 (cofactor formula, same evaluation order) */
    M34 inverse() const
    {
        float det = x00 * (x11 * x22 - x12 * x21) + x10 * (x02 * x21 - x01 * x22) + x20 * (x01 * x12 - x02 * x11);
        if (det == 0.0f)
            throw std::domain_error("can't invert singular matrix");
        float f = 1.0f / det;
        M34 r;
        r.x00 = (x11 * x22 - x12 * x21) * f;
        r.x10 = (x12 * x20 - x10 * x22) * f;
        r.x20 = (x10 * x21 - x11 * x20) * f;
        r.x30 = (-x10 * x21 * x32 + x11 * x20 * x32 + x10 * x22 * x31 - x12 * x20 * x31 - x11 * x22 * x30 +
                 x12 * x21 * x30) *
                f;
        r.x01 = (x02 * x21 - x01 * x22) * f;
        r.x11 = (x00 * x22 - x02 * x20) * f;
        r.x21 = (x01 * x20 - x00 * x21) * f;
        r.x31 = (x00 * x21 * x32 - x01 * x20 * x32 - x00 * x22 * x31 + x02 * x20 * x31 + x01 * x22 * x30 -
                 x02 * x21 * x30) *
                f;
        r.x02 = (x01 * x12 - x02 * x11) * f;
        r.x12 = (x02 * x10 - x00 * x12) * f;
        r.x22 = (x00 * x11 - x01 * x10) * f;
        r.x32 = (-x00 * x11 * x32 + x01 * x10 * x32 + x00 * x12 * x31 - x02 * x10 * x31 - x01 * x12 * x30 +
                 x02 * x11 * x30) *
                f;
        return r;
    }
};

struct Ray
{
    V3 o, d;
    V3 at(float t) const { return o + t * d; } /* ray.h:18-21 */
};

/* ------------------------------------------------------------ textures --- */
struct Img
{
    std::vector<float> px; /* RGBA, row 0 = top */
    unsigned w = 0, h = 0;
    bool valid = false;
    /* Image::getPixel / getPixelAlpha, src/image.cpp:366-395 */
    V3 rgb(int x, int y) const
    {
        if (!valid || y < 0 || (unsigned)y >= h || x < 0 || (unsigned)x >= w)
            return V3();
        const float *p = &px[4 * ((size_t)x + (size_t)y * w)];
        return V3(p[0], p[1], p[2]);
    }
    float alpha(int x, int y) const
    {
        if (!valid || y < 0 || (unsigned)y >= h || x < 0 || (unsigned)x >= w)
            return 0;
        return px[4 * ((size_t)x + (size_t)y * w) + 3];
    }
};

/* Texture evaluations by class on this thread (the op model's texture terms,
 * tools/calibrate_ops.py; SURVEY.md s8(d) counts only geometry and shading) */
enum TexCount { TC_XFORM, TC_MULTIPLY, TC_IMAGE, TC_SPHERICAL, TC_MIRRORBALL, TC_SKYBOX, TC_LOG, TC_N };
thread_local uint64_t tl_tex[TC_N];

struct Tex
{
    virtual ~Tex() {}
    virtual V3 color(V3 p) const = 0;
    /* Texture::getFloat default, texture.h:14-18 */
    virtual float value(V3 p) const
    {
        V3 c = color(p);
        return (c.x + c.y + c.z) * (1.0f / 3.0f);
    }
};

struct ConstTex : Tex
{
    V3 c;
    explicit ConstTex(V3 v) : c(v) {}
    V3 color(V3) const override { return c; }
};

struct CoordTex : Tex
{
    V3 color(V3 p) const override { return p; }
};

/* A user-defined Texture subclass (include/texture.h:10-27): the host functions
 * a test registered for its slot (the same source the product compiles into
 * the device module through pt_tex_device, built here with -ffp-contract=off) */
typedef void (*user_color_fn)(const float *p, const float *prm, float *out);
typedef float (*user_value_fn)(const float *p, const float *prm);
struct UserFns
{
    user_color_fn color = nullptr;
    user_value_fn value = nullptr;
};
std::map<int, UserFns> &user_slots()
{
    static std::map<int, UserFns> m;
    return m;
}
struct UserTex : Tex
{
    UserFns fn;
    std::vector<float> prm;
    V3 color(V3 p) const override
    {
        const float q[3] = {p.x, p.y, p.z};
        float o[3];
        fn.color(q, prm.data(), o);
        return V3(o[0], o[1], o[2]);
    }
    float value(V3 p) const override
    {
        if (!fn.value)
            return Tex::value(p);
        const float q[3] = {p.x, p.y, p.z};
        return fn.value(q, prm.data());
    }
};

struct XformTex : Tex /* TransformedTexture, texture.h:60-90 */
{
    M34 m;
    std::unique_ptr<Tex> t;
    V3 color(V3 p) const override { return tl_tex[TC_XFORM]++, t->color(m.apply(p)); }
    float value(V3 p) const override { return tl_tex[TC_XFORM]++, t->value(m.apply(p)); }
};

/* nearest-texel lookup of ImageTexture / ImageAlphaTexture (image_texture.h:18-28, :44-65):
 * `x -= floor(x)` calls ::floor(double); the difference is exact in float either way. */
inline void planar_texel(const Img &im, V3 v, int &xi, int &yi)
{
    tl_tex[TC_IMAGE]++;
    float x = v.x, y = v.y;
    x = (float)((double)x - ::floor((double)x));
    y = (float)((double)y - ::floor((double)y));
    y = 1 - y;
    x *= (float)im.w;
    y *= (float)im.h;
    xi = (int)std::floor(x);
    yi = (int)std::floor(y);
}

struct ImageTex : Tex
{
    const Img *im;
    V3 color(V3 v) const override
    {
        int xi, yi;
        planar_texel(*im, v, xi, yi);
        return im->rgb(xi, yi);
    }
};

struct ImageAlphaTex : Tex
{
    const Img *im;
    V3 color(V3 v) const override
    {
        int xi, yi;
        planar_texel(*im, v, xi, yi);
        return V3(im->alpha(xi, yi));
    }
    float value(V3 v) const override
    {
        int xi, yi;
        planar_texel(*im, v, xi, yi);
        return im->alpha(xi, yi);
    }
};

/* Cube-face selection shared by both skybox textures (image_texture.h:90-110,
 * :135-176): returns the face index and its (x, y) in [-1, 1]. */
inline int skybox_face(V3 v, float &fx, float &fy)
{
    V3 a(std::fabs(v.x), std::fabs(v.y), std::fabs(v.z));
    enum { TOP, BOTTOM, LEFT, RIGHT, FRONT, BACK };
    if (a.x > a.y && a.x > a.z) {
        if (v.x < 0) {
            fx = -v.z / a.x, fy = v.y / a.x;
            return LEFT;
        }
        fx = v.z / a.x, fy = v.y / a.x;
        return RIGHT;
    }
    if (a.y > a.z) {
        if (v.y < 0) {
            fx = -v.x / a.y, fy = v.z / a.y;
            return BOTTOM;
        }
        fx = v.x / a.y, fy = v.z / a.y;
        return TOP;
    }
    if (v.z < 0) {
        fx = v.x / a.z, fy = v.y / a.z;
        return BACK;
    }
    fx = -v.x / a.z, fy = v.y / a.z;
    return FRONT;
}

inline void skybox_texel(const Img &im, float x, float y, int &xi, int &yi)
{
    x = (float)(x * 0.5 + 0.5);
    y = (float)(0.5 - y * 0.5);
    x *= (float)im.w;
    y *= (float)im.h;
    xi = (int)std::floor(x);
    yi = (int)std::floor(y);
}

struct SkyboxTex : Tex
{
    const Img *face[6]; /* top bottom left right front back */
    bool alpha = false;
    float lookup(V3 v, bool want_alpha, V3 &rgb) const
    {
        tl_tex[TC_SKYBOX]++;
        float fx, fy;
        int f = skybox_face(v, fx, fy);
        int xi, yi;
        skybox_texel(*face[f], fx, fy, xi, yi);
        if (want_alpha)
            return face[f]->alpha(xi, yi);
        rgb = face[f]->rgb(xi, yi);
        return 0;
    }
    V3 color(V3 v) const override
    {
        if (v == V3(0))
            return V3(0);
        V3 rgb;
        if (alpha)
            return V3(lookup(v, true, rgb));
        lookup(v, false, rgb);
        return rgb;
    }
    float value(V3 v) const override
    {
        if (!alpha)
            return Tex::value(v);
        if (v == V3(0))
            return 0;
        V3 rgb;
        return lookup(v, true, rgb);
    }
};

struct MultiplyTex : Tex /* filter_texture.h:36-56 */
{
    V3 f;
    std::unique_ptr<Tex> t;
    V3 color(V3 p) const override { return tl_tex[TC_MULTIPLY]++, t->color(p) * f; }
};

struct LogTex : Tex /* filter_texture.h:58-82 */
{
    std::unique_ptr<Tex> t;
    static float lg(float v)
    {
        if ((double)v <= 1e-30)
            return 0;
        return 0.5f + std::log(v) / (float)::log(2.0) / 256;
    }
    V3 color(V3 p) const override
    {
        tl_tex[TC_LOG]++;
        V3 c = t->color(p);
        return V3(lg(c.x), lg(c.y), lg(c.z));
    }
};

struct MirrorBallTex : Tex /* transform_texture.h:33-59 */
{
    std::unique_ptr<Tex> t;
    static V3 map(V3 v)
    {
        tl_tex[TC_MIRRORBALL]++;
        if (v == V3(0))
            return V3(0);
        v = normalize(v);
        if (v.z <= -1)
            return V3(0, 0.5f, 0);
        float d = std::sqrt(2 + 2 * v.z);
        if (d == 0)
            return V3(0, 0.5f, 0);
        float xt = v.x / d, yt = v.y / d;
        return V3((float)(xt * 0.5 + 0.5), (float)(yt * 0.5 + 0.5), 0);
    }
    V3 color(V3 p) const override { return t->color(map(p)); }
    float value(V3 p) const override { return t->value(map(p)); }
};

/* transform_texture.h:61-85.  atan2f; and `asin(v.z)` on a float is asinf:
 * src/test.cpp:22 includes image_texture.h -> image.h:28 (`using namespace std;`
 * at global scope) before transform_texture.h, so std::asin(float) wins
 * overload resolution in the reference's translation unit. */
struct SphericalTex : Tex
{
    std::unique_ptr<Tex> t;
    static V3 map(V3 v)
    {
        tl_tex[TC_SPHERICAL]++;
        if (v == V3(0))
            return V3(0);
        v = normalize(v);
        float theta = std::atan2(v.y, v.x);
        if (theta < -M_PI)
            theta = (float)(theta + 2 * M_PI);
        if (theta > M_PI)
            theta = (float)(theta - 2 * M_PI);
        float phi = std::asin(v.z);
        return V3((float)(theta * 0.5 / M_PI + 0.5), (float)(phi / (M_PI / 2) * 0.5 + 0.5), 0);
    }
    V3 color(V3 p) const override { return t->color(map(p)); }
    float value(V3 p) const override { return t->value(map(p)); }
};

struct Material /* include/material.h:10-37 */
{
    std::unique_ptr<Tex> reflect, scatter, emissive, transmit, trc;
    float ior = 1;
    int id = -1;
};

/* ------------------------------------------------------------ geometry --- */
struct Span /* include/span.h:12-120 */
{
    float t0;
    V3 n0;
    const Material *m0;
    float t1;
    V3 n1;
    const Material *m1;
    void start_from_start(const Span &s) { t0 = s.t0, m0 = s.m0, n0 = s.n0; }
    void end_from_start(const Span &s) { t1 = s.t0, m1 = s.m0, n1 = -s.n0; }
    void start_from_end(const Span &s) { t0 = s.t1, m0 = s.m1, n0 = -s.n1; }
    void end_from_end(const Span &s) { t1 = s.t1, m1 = s.m1, n1 = s.n1; }
};

struct SpanList
{
    std::vector<Span> v;
    void push(const Span &s)
    {
        if (v.size() > 100000)
            throw std::runtime_error("runaway span list");
        v.push_back(s);
    }
};

struct Stats
{
    uint64_t queries = 0, sphere_tests = 0, sphere_hits = 0, plane_tests = 0, merge_steps = 0, shaded = 0,
             refract_children = 0, scatter_children = 0, attempts = 0, draws = 0, leaf_children = 0;
    uint64_t tex[7] = {0, 0, 0, 0, 0, 0, 0}; /* texture evaluations by class (TexCount) */
    void add(const Stats &o)
    {
        for (int k = 0; k < 7; k++) tex[k] += o.tex[k];
        queries += o.queries, sphere_tests += o.sphere_tests, sphere_hits += o.sphere_hits;
        plane_tests += o.plane_tests, merge_steps += o.merge_steps, shaded += o.shaded;
        refract_children += o.refract_children, scatter_children += o.scatter_children;
        attempts += o.attempts, draws += o.draws, leaf_children += o.leaf_children;
    }
};

struct Node
{
    virtual ~Node() {}
    virtual void spans(const Ray &r, SpanList &out, Stats &st) const = 0;
};

struct SphereNode : Node /* src/sphere.cpp:6-49 */
{
    V3 c;
    float r2;
    const Material *m;
    void spans(const Ray &r, SpanList &out, Stats &st) const override
    {
        st.sphere_tests++;
        V3 oc = r.o - c;
        float a = dot(r.d, r.d);
        float b = dot(oc, r.d);
        float cc = dot(oc, oc) - r2;
        float disc = b * b - a * cc;
        if (disc <= kEps)
            return;
        st.sphere_hits++;
        float s = std::sqrt(disc);
        Span sp;
        sp.t0 = (-b - s) / a;
        sp.t1 = (-b + s) / a;
        sp.n0 = normalize(r.at(sp.t0) - c);
        sp.n1 = normalize(r.at(sp.t1) - c);
        sp.m0 = sp.m1 = m;
        out.push(sp);
    }
};

/* A user-defined Object subclass with one span per ray (pt_object_device):
 * the host functions a test registered for its slot (the same source the
 * product compiles into the device module, built with -ffp-contract=off). */
typedef int (*user_span_fn)(const float *o, const float *d, const float *prm, float *t01);
typedef void (*user_normal_fn)(const float *p, const float *prm, float *n);
struct UserObjFns
{
    user_span_fn span = nullptr;
    user_normal_fn normal = nullptr;
};
std::map<int, UserObjFns> &user_obj_slots()
{
    static std::map<int, UserObjFns> m;
    return m;
}
struct UserNode : Node
{
    UserObjFns fn;
    std::vector<float> prm;
    const Material *m;
    V3 normal(V3 p) const
    {
        const float q[3] = {p.x, p.y, p.z};
        float n[3];
        fn.normal(q, prm.data(), n);
        return V3(n[0], n[1], n[2]);
    }
    void spans(const Ray &r, SpanList &out, Stats &) const override
    {
        const float o[3] = {r.o.x, r.o.y, r.o.z}, d[3] = {r.d.x, r.d.y, r.d.z};
        float t[2];
        if (!fn.span(o, d, prm.data(), t))
            return;
        Span sp;
        sp.t0 = t[0], sp.t1 = t[1];
        sp.n0 = normal(r.at(sp.t0));
        sp.n1 = normal(r.at(sp.t1));
        sp.m0 = sp.m1 = m;
        out.push(sp);
    }
};

struct PlaneNode : Node /* src/plane.cpp:23-63: half-space {p : n.p + d < 0} */
{
    V3 n;
    float d;
    const Material *m;
    void spans(const Ray &r, SpanList &out, Stats &st) const override
    {
        st.plane_tests++;
        float div = dot(r.d, n);
        float num = -d - dot(r.o, n);
        Span sp;
        sp.n0 = sp.n1 = normalize(n);
        sp.m0 = sp.m1 = m;
        float t = 0;
        bool degenerate = std::fabs(div) < kEps * kEps;
        if (!degenerate) {
            t = num / div;
            degenerate = std::fabs(t) >= kMaxValue;
        }
        if (degenerate) {
            if (std::fabs(num) < kEps * kEps) {
                sp.t0 = -kMaxValue;
                sp.t1 = kMaxValue;
                out.push(sp);
            }
        } else if (div < 0) {
            sp.t0 = t;
            sp.t1 = kMaxValue;
            out.push(sp);
        } else {
            sp.t0 = -kMaxValue;
            sp.t1 = t;
            out.push(sp);
        }
    }
};

/* Two-way merges over complete child lists; each loop body is the reference's
 * next() with nextA()/nextB() = "pull the next element or mark ended". */
struct Cursor
{
    const std::vector<Span> *v;
    size_t i = 0;
    Span cur;
    bool ended = false;
    explicit Cursor(const std::vector<Span> &l) : v(&l) { pull(); }
    void pull()
    {
        if (i < v->size())
            cur = (*v)[i++];
        else
            ended = true;
    }
};

struct UnionNode : Node /* src/union.cpp:84-134 */
{
    std::unique_ptr<Node> a, b;
    void spans(const Ray &r, SpanList &out, Stats &st) const override
    {
        SpanList la, lb;
        a->spans(r, la, st);
        b->spans(r, lb, st);
        Cursor A(la.v), B(lb.v);
        for (;;) {
            st.merge_steps++;
            if (A.ended) {
                if (B.ended)
                    return;
                out.push(B.cur), B.pull();
            } else if (B.ended) {
                out.push(A.cur), A.pull();
            } else if (A.cur.t1 < B.cur.t0) {
                out.push(A.cur), A.pull();
            } else if (B.cur.t1 < A.cur.t0) {
                out.push(B.cur), B.pull();
            } else if (A.cur.t0 < B.cur.t0) {
                if (A.cur.t1 < B.cur.t1)
                    A.cur.end_from_end(B.cur);
                B.pull();
            } else {
                if (A.cur.t1 > B.cur.t1)
                    B.cur.end_from_end(A.cur);
                A.pull();
            }
        }
    }
};

struct IntersectionNode : Node /* src/intersection.cpp:84-130 */
{
    std::unique_ptr<Node> a, b;
    void spans(const Ray &r, SpanList &out, Stats &st) const override
    {
        SpanList la, lb;
        a->spans(r, la, st);
        b->spans(r, lb, st);
        Cursor A(la.v), B(lb.v);
        for (;;) {
            st.merge_steps++;
            if (A.ended || B.ended)
                return;
            if (A.cur.t1 < B.cur.t0) {
                A.pull();
            } else if (B.cur.t1 < A.cur.t0) {
                B.pull();
            } else if (A.cur.t0 < B.cur.t0) {
                if (A.cur.t1 < B.cur.t1) {
                    A.cur.start_from_start(B.cur);
                    out.push(A.cur), A.pull();
                } else {
                    out.push(B.cur), B.pull();
                }
            } else {
                if (B.cur.t1 < A.cur.t1) {
                    B.cur.start_from_start(A.cur);
                    out.push(B.cur), B.pull();
                } else {
                    out.push(A.cur), A.pull();
                }
            }
        }
    }
};

struct DifferenceNode : Node /* src/difference.cpp:84-135, including the :124-130 quirk */
{
    std::unique_ptr<Node> a, b;
    void spans(const Ray &r, SpanList &out, Stats &st) const override
    {
        SpanList la, lb;
        a->spans(r, la, st);
        b->spans(r, lb, st);
        Cursor A(la.v), B(lb.v);
        for (;;) {
            st.merge_steps++;
            if (A.ended)
                return;
            if (B.ended) {
                out.push(A.cur), A.pull();
            } else if (A.cur.t1 < B.cur.t0) {
                out.push(A.cur), A.pull();
            } else if (B.cur.t1 < A.cur.t0) {
                B.pull();
            } else if (A.cur.t0 < B.cur.t0) {
                if (A.cur.t1 < B.cur.t1) {
                    A.cur.end_from_start(B.cur);
                    out.push(A.cur), A.pull();
                } else {
                    Span res = A.cur;
                    res.end_from_start(B.cur);
                    A.cur.start_from_end(B.cur);
                    B.pull();
                    out.push(res);
                }
            } else if (A.cur.t1 > B.cur.t1) {
                A.cur.end_from_start(B.cur); /* sic: reference calls copyEndFromStart here */
                B.pull();
            } else {
                A.pull();
            }
        }
    }
};

struct XformNode : Node /* TransformedObject, include/object.h:26-76 */
{
    M34 m, inv;
    std::unique_ptr<Node> c;
    void spans(const Ray &r, SpanList &out, Stats &st) const override
    {
        Ray lr{m.apply(r.o), m.apply_linear(r.d)};
        SpanList l;
        c->spans(lr, l, st);
        for (Span s : l.v) {
            s.n0 = normalize(inv.apply_linear(s.n0));
            s.n1 = normalize(inv.apply_linear(s.n1));
            out.push(s);
        }
    }
};

/* --------------------------------------------------------------- scene --- */
struct Scene
{
    std::map<int, std::unique_ptr<Img>> images;
    std::map<int, std::unique_ptr<Material>> mats;
    std::unique_ptr<Node> root;
};

std::vector<char> slurp(const std::string &p)
{
    std::ifstream f(p, std::ios::binary);
    if (!f)
        throw std::runtime_error("cannot open " + p);
    return std::vector<char>((std::istreambuf_iterator<char>(f)), std::istreambuf_iterator<char>());
}

std::unique_ptr<Tex> make_tex(const scenetext::Desc &d, Scene &s, int id)
{
    const scenetext::Item &t = scenetext::find(d.textures, id, "texture");
    auto img = [&](int k) -> const Img * { return s.images.at(t.i[k]).get(); };
    if (t.type == "color")
        return std::unique_ptr<Tex>(new ConstTex(V3(t.f[0], t.f[1], t.f[2])));
    if (t.type == "coord")
        return std::unique_ptr<Tex>(new CoordTex());
    if (t.type == "user") {
        auto it = user_slots().find(t.i[0]);
        if (it == user_slots().end() || !it->second.color)
            throw std::runtime_error("oracle: no host function registered for user texture slot " +
                                     std::to_string(t.i[0]));
        auto p = new UserTex;
        p->fn = it->second;
        p->prm = t.f;
        return std::unique_ptr<Tex>(p);
    }
    if (t.type == "image") {
        auto p = new ImageTex;
        p->im = img(0);
        return std::unique_ptr<Tex>(p);
    }
    if (t.type == "image_alpha") {
        auto p = new ImageAlphaTex;
        p->im = img(0);
        return std::unique_ptr<Tex>(p);
    }
    if (t.type == "skybox" || t.type == "skybox_alpha") {
        auto p = new SkyboxTex;
        for (int k = 0; k < 6; k++) p->face[k] = img(k);
        p->alpha = t.type == "skybox_alpha";
        return std::unique_ptr<Tex>(p);
    }
    if (t.type == "multiply") {
        auto p = new MultiplyTex;
        p->f = V3(t.f[0], t.f[1], t.f[2]);
        p->t = make_tex(d, s, t.i[0]);
        return std::unique_ptr<Tex>(p);
    }
    if (t.type == "log") {
        auto p = new LogTex;
        p->t = make_tex(d, s, t.i[0]);
        return std::unique_ptr<Tex>(p);
    }
    if (t.type == "mirrorball") {
        auto p = new MirrorBallTex;
        p->t = make_tex(d, s, t.i[0]);
        return std::unique_ptr<Tex>(p);
    }
    if (t.type == "spherical") {
        auto p = new SphericalTex;
        p->t = make_tex(d, s, t.i[0]);
        return std::unique_ptr<Tex>(p);
    }
    if (t.type == "xform") {
        auto p = new XformTex;
        p->m = M34::from(t.f.data());
        p->t = make_tex(d, s, t.i[0]);
        return std::unique_ptr<Tex>(p);
    }
    throw std::runtime_error("oracle: unknown texture " + t.type);
}

std::unique_ptr<Node> make_node(const scenetext::Desc &d, Scene &s, int id)
{
    const scenetext::Item &o = scenetext::find(d.objects, id, "object");
    if (o.type == "sphere") {
        auto p = new SphereNode;
        p->c = V3(o.f[0], o.f[1], o.f[2]);
        p->r2 = o.f[3] * o.f[3]; /* sphere.cpp:10 */
        p->m = s.mats.at(o.i[0]).get();
        return std::unique_ptr<Node>(p);
    }
    if (o.type == "plane") {
        auto p = new PlaneNode;
        p->n = V3(o.f[0], o.f[1], o.f[2]);
        p->d = o.f[3];
        p->m = s.mats.at(o.i[0]).get();
        return std::unique_ptr<Node>(p);
    }
    if (o.type == "user") {
        auto it = user_obj_slots().find(o.i[1]);
        if (it == user_obj_slots().end() || !it->second.span || !it->second.normal)
            throw std::runtime_error("oracle: no host functions registered for user object slot " +
                                     std::to_string(o.i[1]));
        auto p = new UserNode;
        p->fn = it->second;
        p->prm = o.f;
        p->m = s.mats.at(o.i[0]).get();
        return std::unique_ptr<Node>(p);
    }
    if (o.type == "union") {
        auto p = new UnionNode;
        p->a = make_node(d, s, o.i[0]);
        p->b = make_node(d, s, o.i[1]);
        return std::unique_ptr<Node>(p);
    }
    if (o.type == "intersection") {
        auto p = new IntersectionNode;
        p->a = make_node(d, s, o.i[0]);
        p->b = make_node(d, s, o.i[1]);
        return std::unique_ptr<Node>(p);
    }
    if (o.type == "difference") {
        auto p = new DifferenceNode;
        p->a = make_node(d, s, o.i[0]);
        p->b = make_node(d, s, o.i[1]);
        return std::unique_ptr<Node>(p);
    }
    if (o.type == "xform") {
        auto p = new XformNode;
        p->m = M34::from(o.f.data());
        p->inv = p->m.inverse();
        p->c = make_node(d, s, o.i[0]);
        return std::unique_ptr<Node>(p);
    }
    throw std::runtime_error("oracle: unknown object " + o.type);
}

std::unique_ptr<Scene> load_scene(const std::string &text)
{
    scenetext::Desc d = scenetext::parse(text);
    std::unique_ptr<Scene> s(new Scene);
    for (const scenetext::Item &im : d.images) {
        if (im.type != "raw")
            throw std::runtime_error("oracle: only raw RGBA32F images are supported");
        std::unique_ptr<Img> img(new Img);
        img->w = im.i[0];
        img->h = im.i[1];
        std::vector<char> raw = slurp(im.path);
        if (raw.size() != (size_t)img->w * img->h * 16)
            throw std::runtime_error("oracle: raw image size mismatch");
        img->px.resize(raw.size() / 4);
        memcpy(img->px.data(), raw.data(), raw.size());
        img->valid = true;
        s->images[im.id] = std::move(img);
    }
    for (const scenetext::Item &m : d.materials) {
        std::unique_ptr<Material> mat(new Material);
        mat->reflect = make_tex(d, *s, m.i[0]);
        mat->scatter = make_tex(d, *s, m.i[1]);
        mat->emissive = make_tex(d, *s, m.i[2]);
        mat->transmit = make_tex(d, *s, m.i[3]);
        mat->trc = make_tex(d, *s, m.i[4]);
        mat->ior = m.f[0];
        mat->id = m.id;
        s->mats[m.id] = std::move(mat);
    }
    s->root = make_node(d, *s, d.root);
    return s;
}

/* -------------------------------------------------------------- tracer --- */
enum Order { ORDER_REFERENCE = 0, ORDER_FAST = 1 };

/* uniform_real_distribution<float>::operator(), vector3d.h:22-33 */
template <class E>
inline float uniform(E &e, float lo, float hi)
{
    float r = (float)e();
    r -= (float)(int64_t)E::min();
    r /= (float)((int64_t)E::max() - (int64_t)E::min());
    r *= hi - lo;
    r += lo;
    return r;
}

inline float clamp01(float x)
{
    float m = (x < 1.0f) ? x : 1.0f; /* std::min(1.0f, x) */
    return (0.0f < m) ? m : 0.0f;    /* std::max(0.0f, m) */
}

/* pairwise tree over 64 slots padded with -0.0f (x + -0.0f == x for every x) */
inline V3 pairwise64(const std::vector<V3> &g)
{
    float b[3][64];
    for (int k = 0; k < 64; k++) {
        V3 v = k < (int)g.size() ? g[k] : V3(-0.0f, -0.0f, -0.0f);
        b[0][k] = v.x, b[1][k] = v.y, b[2][k] = v.z;
    }
    for (int w = 1; w < 64; w *= 2)
        for (int k = 0; k < 64; k += 2 * w)
            for (int c = 0; c < 3; c++) b[c][k] = b[c][k] + b[c][k + w];
    return V3(b[0][0], b[1][0], b[2][0]);
}

/* The fast order's run of leaf children (ORDER_FAST above): non-zero terms
 * dealt round-robin to 64 lane sums, flushed into retval as their pairwise
 * tree.  An empty run adds nothing. */
struct LaneSums
{
    float l[3][64];
    int nz = 0, len = 0;
    LaneSums() { reset(); }
    void reset()
    {
        for (int c = 0; c < 3; c++)
            for (int k = 0; k < 64; k++) l[c][k] = 0.0f;
        nz = len = 0;
    }
    void add(V3 t)
    {
        len++;
        if (t.x == 0.0f && t.y == 0.0f && t.z == 0.0f)
            return;
        const int k = nz++ & 63;
        l[0][k] = l[0][k] + t.x, l[1][k] = l[1][k] + t.y, l[2][k] = l[2][k] + t.z;
    }
    void flush(V3 &retval)
    {
        if (!len)
            return;
        std::vector<V3> g(64);
        for (int k = 0; k < 64; k++) g[k] = V3(l[0][k], l[1][k], l[2][k]);
        retval = retval + pairwise64(g);
        reset();
    }
};

/* A pixel's sum of spp samples: in the reference order one after the other
 * (tracePixel, path-trace.h:192-199); in the group-64 order in blocks of 32
 * consecutive samples, each block its pairwise tree (missing leaves -0.0f),
 * the block sums added one after the other -- the GPU fast path's pixel sum
 * (pt_device.h pt_reduce / render_chunk block partials). */
template <class F>
V3 pixel_sum(int spp, int order, F &&sample)
{
    V3 acc(0, 0, 0);
    if (order != ORDER_FAST) {
        for (int s = 0; s < spp; s++) acc = acc + sample(s);
        return acc;
    }
    std::vector<V3> blk;
    blk.reserve(32);
    for (int s = 0; s < spp; s++) {
        blk.push_back(sample(s));
        if (blk.size() == 32 || s == spp - 1) {
            acc = acc + pairwise64(blk);
            blk.clear();
        }
    }
    return acc;
}

template <class E>
struct Tracer
{
    const Scene &scene;
    Order order;
    Stats st;
    Tracer(const Scene &s, Order o) : scene(s), order(o) {}

    float u(E &e, float lo, float hi)
    {
        st.draws++;
        return uniform(e, lo, hi);
    }

    /* Vector3D::rand(r, 1, 0), vector3d.h:163-185 */
    V3 rand_ball(E &e)
    {
        V3 v;
        float mag;
        do {
            st.attempts++;
            v.x = u(e, -1, 1);
            v.y = u(e, -1, 1);
            v.z = u(e, -1, 1);
            mag = length(v);
        } while (mag > 1);
        return v;
    }

    /* traceRay<T>, include/path-trace.h:58-165 */
    V3 trace(const Ray &ray, int depth, E &rng, float strength)
    {
        st.queries++;
        SpanList l;
        scene.root->spans(ray, l, st);
        float t = -1;
        const Material *mat = nullptr;
        V3 n;
        float ior = 1;
        for (const Span &s : l.v) {
            if (s.t0 >= kMaxValue)
                return V3(0, 0, 0);
            if (s.t0 >= kEps) {
                t = s.t0, n = s.n0, mat = s.m0;
                ior = (float)(1.0 / (double)mat->ior);
                break;
            }
            if (s.t1 >= kMaxValue)
                return V3(0, 0, 0);
            if (s.t1 >= kEps) {
                t = s.t1, n = -s.n1, mat = s.m1;
                ior = mat->ior;
                break;
            }
        }
        if (t == -1)
            return V3(0, 0, 0);
        V3 hit = ray.at(t);
        V3 retval = mat->emissive->color(hit);
        float addFactor = 1;
        if (depth <= 0 || strength < kEps)
            return retval;
        st.shaded++;
        float rf = clamp01(mat->trc->value(hit)) * refract_strength(ray.d, ior, n);
        if (rf > kEps) {
            V3 rd = refract(ray.d, ior, n);
            if (rd != V3(0, 0, 0)) {
                V3 tr = mat->transmit->color(hit);
                st.refract_children++;
                V3 w = addFactor * rf * tr;
                retval = retval + w * trace(Ray{hit, rd}, depth - 1, rng, strength * rf * addFactor * length(tr));
                addFactor *= 1 - rf;
            }
        }
        if (addFactor < kEps)
            return retval;
        float sc = clamp01(mat->scatter->value(hit));
        int N = (int)(10000 * strength * addFactor * sc);
        if (sc <= kEps)
            N = 1;
        if (N == 0)
            N = 1;
        V3 rc = mat->reflect->color(hit);
        LaneSums run;
        bool grouped = order == ORDER_FAST && sc > kEps;
        for (int i = 0; i < N; i++) {
            V3 refl = reflect(ray.d, n);
            V3 dir = refl;
            if (sc > kEps) {
                int count = 0;
                do {
                    count++;
                    if (count > 1000) { /* path-trace.h:148-152 (NDEBUG semantics) */
                        run.flush(retval);
                        return retval;
                    }
                    dir = rand_ball(rng);
                    dir = dir + (1 / sc - 1) * refl;
                } while (dot(n, dir) <= kEps);
                dir = normalize(dir);
            }
            float factor = 1 - (1 - dot(dir, n)) * sc;
            float cs = strength / N * addFactor * factor * length(rc);
            V3 w = addFactor / N * factor * rc;
            st.scatter_children++;
            bool leaf = depth - 1 <= 0 || cs < kEps;
            if (leaf)
                st.leaf_children++;
            V3 child = trace(Ray{ray.at(t), dir}, depth - 1, rng, cs);
            if (grouped && leaf) {
                run.add(w * child);
            } else {
                run.flush(retval);
                retval = retval + w * child;
            }
        }
        run.flush(retval);
        return retval;
    }

    /* one sample of tracePixel<T>(int px, ...), path-trace.h:187-201 with spp = 1 */
    V3 sample(int px, int py, int W, int H, int depth, float sw, float sh, float dist, E &rng)
    {
        float x = 2 * (px + u(rng, 0, 1)) / W - 1;
        float y = 1 - 2 * (py + u(rng, 0, 1)) / H;
        Ray r{V3(0, 0, 0), V3(x * sw, y * sh, -dist)};
        V3 c = V3(0, 0, 0) + trace(r, depth, rng, 1.0f);
        return c / (float)1;
    }
};

thread_local std::string g_err;

} // namespace oracle

using namespace oracle;

extern "C" {

const char *oracle_last_error() { return g_err.c_str(); }

/* test infrastructure: the host functions of user object slot `slot` */
int oracle_register_user_object(int slot, user_span_fn span, user_normal_fn normal)
{
    if (!span || !normal)
        return -1;
    user_obj_slots()[slot] = UserObjFns{span, normal};
    return 0;
}

/* test infrastructure: the host functions of user texture slot `slot` (value may be NULL) */
int oracle_register_user_texture(int slot, user_color_fn color, user_value_fn value)
{
    if (!color)
        return -1;
    user_slots()[slot] = UserFns{color, value};
    return 0;
}

} // extern "C"

namespace oracle
{
/* RenderBlock (reference src/test.cpp:324-507) restated depth-first as the
 * reference runs it: calcPixelColor :441-465, interpolateSquare :423-436,
 * colorCloseEnough :437-440, renderSquare :466-499, run :501-507,
 * copyToBuffer :362-374.  tracePixel = spp samples of the per-(pixel, sample)
 * engine keyed by py * gw + px, gw = ceil(W / block) * block + 1 (block
 * corners reach past the right edge), summed in order, / spp. */
struct AdaptiveBlock
{
    int x0, y0, S, W, H, maxS;
    float mcd;
    std::vector<V3> buf;
    std::vector<char> valid;
    std::function<V3(int, int)> trace_pixel;
    bool in(int x, int y) const { return !(x < x0 || x - x0 > S) && !(y < y0 || y - y0 > S); }
    size_t at(int x, int y) const { return (size_t)(x - x0) + (size_t)(y - y0) * (S + 1); }
    void set_pixel(int x, int y, V3 c)
    {
        if (!in(x, y))
            return;
        buf[at(x, y)] = c;
        valid[at(x, y)] = 1;
    }
    V3 calc(int x, int y)
    {
        if (x >= x0 && x <= x0 + S && y >= y0 && y <= y0 + S && valid[at(x, y)])
            return buf[at(x, y)];
        V3 r = trace_pixel(x, y);
        set_pixel(x, y, r);
        return r;
    }
    bool close(V3 a, V3 b) const { return dot(a - b, a - b) <= mcd * mcd * dot(a, a); }
    void interpolate(int xo, int yo, int size, V3 tl, V3 tr, V3 bl, V3 br)
    {
        for (int y = 0; y < size; y++) {
            float fy = (float)y / size;
            V3 l = tl + fy * (bl - tl);
            V3 r = tr + fy * (br - tr);
            for (int x = 0; x < size; x++) {
                float fx = (float)x / size;
                set_pixel(x + xo, y + yo, l + fx * (r - l));
            }
        }
    }
    void square(int x, int y, int size, V3 tl, V3 tr, V3 bl, V3 br)
    {
        if (x > W || y > H)
            return;
        if (size <= 1) {
            set_pixel(x, y, tl);
            return;
        }
        if (close(tl, tr) && close(tl, bl) && close(tl, br) && close(tr, bl) && close(tr, br) && close(bl, br) &&
            size <= maxS) {
            interpolate(x, y, size, tl, tr, bl, br);
            return;
        }
        int half = size / 2, cx = x + half, cy = y + half;
        V3 tc = calc(cx, y);
        V3 cl = calc(x, cy);
        V3 cc = calc(cx, cy);
        V3 cr = calc(x + size, cy);
        V3 bc = calc(cx, y + size);
        square(x, y, half, tl, tc, cl, cc);
        square(cx, y, half, tc, tr, cc, cr);
        square(x, cy, half, cl, cc, bl, bc);
        square(cx, cy, half, cc, cr, bc, br);
    }
    void run()
    {
        V3 tl = calc(x0, y0), tr = calc(x0 + S, y0), bl = calc(x0, y0 + S), br = calc(x0 + S, y0 + S);
        square(x0, y0, S, tl, tr, bl, br);
    }
};
} // namespace oracle

extern "C" {

/* out: W*H*3; traced (optional): number of tracePixel calls (cache misses) */
int oracle_render_adaptive(const char *scene_text, int W, int H, int spp, int depth, float sw, float sh, float dist,
                           uint64_t seed, int block, int max_interp, float min_delta, int threads, int order,
                           float *out, uint64_t *traced)
{
    try {
        std::unique_ptr<Scene> scene = load_scene(scene_text);
        const int gw = (W + block - 1) / block * block + 1; /* blocks reach x = ceil(W / block) * block */
        std::vector<std::pair<int, int>> origins;
        for (int y0 = 0; y0 < H; y0 += block)
            for (int x0 = 0; x0 < W; x0 += block) origins.push_back({x0, y0});
        std::fill(out, out + (size_t)W * H * 3, 0.0f);
        std::atomic<int> next(0);
        std::atomic<uint64_t> ntraced(0);
        std::mutex mu;
        std::string err;
        auto worker = [&]() {
            Tracer<SampleEngine> tr(*scene, order == 1 ? ORDER_FAST : ORDER_REFERENCE);
            try {
                for (;;) {
                    int k = next.fetch_add(1);
                    if (k >= (int)origins.size())
                        break;
                    AdaptiveBlock b;
                    b.x0 = origins[k].first, b.y0 = origins[k].second, b.S = block, b.W = W, b.H = H;
                    b.maxS = max_interp, b.mcd = min_delta;
                    b.buf.assign((size_t)(block + 1) * (block + 1), V3(0, 0, 0));
                    b.valid.assign((size_t)(block + 1) * (block + 1), 0);
                    b.trace_pixel = [&](int px, int py) {
                        const uint64_t p = (uint64_t)py * gw + px;
                        V3 acc = pixel_sum(spp, order == 1 ? ORDER_FAST : ORDER_REFERENCE, [&](int s) {
                            SampleEngine e(seed, p, (uint64_t)s);
                            return tr.sample(px, py, W, H, depth, sw, sh, dist, e);
                        });
                        ntraced++;
                        return acc / (float)spp;
                    };
                    b.run();
                    for (int y = b.y0; y < b.y0 + block && y < H; y++)
                        for (int x = b.x0; x < b.x0 + block && x < W; x++)
                            if (b.valid[b.at(x, y)]) {
                                V3 c = b.buf[b.at(x, y)];
                                float *o = out + 3 * ((size_t)y * W + x);
                                o[0] = c.x, o[1] = c.y, o[2] = c.z;
                            }
                }
            } catch (std::exception &e) {
                std::lock_guard<std::mutex> g(mu);
                err = e.what();
            }
        };
        std::vector<std::thread> pool;
        for (int t = 0; t < (threads < 1 ? 1 : threads); t++) pool.emplace_back(worker);
        for (auto &t : pool) t.join();
        if (!err.empty())
            throw std::runtime_error(err);
        if (traced)
            *traced = ntraced.load();
        return 0;
    } catch (std::exception &e) {
        g_err = e.what();
        return -1;
    }
}


/* stats[0..10]: queries sphere_tests sphere_hits plane_tests merge_steps shaded
 * refract_children scatter_children attempts draws leaf_children; stats[11..17]:
 * texture evaluations (TexCount: xform multiply image spherical mirrorball
 * skybox log) -- the caller's array holds 18 */
int oracle_render_gw(const char *scene_text, int W, int H, int gw, int spp, int depth, float sw, float sh,
                     float dist, uint64_t seed, const int32_t *pixels, int npx, int threads, int order,
                     int per_sample, float *out, uint64_t *stats);

int oracle_render(const char *scene_text, int W, int H, int spp, int depth, float sw, float sh, float dist,
                  uint64_t seed, const int32_t *pixels, int npx, int threads, int order, int per_sample, float *out,
                  uint64_t *stats)
{
    return oracle_render_gw(scene_text, W, H, W, spp, depth, sw, sh, dist, seed, pixels, npx, threads, order,
                            per_sample, out, stats);
}

/* pixel index p = py * gw + px (gw = W, or W + 1 for the adaptive caller) */
int oracle_render_gw(const char *scene_text, int W, int H, int gw, int spp, int depth, float sw, float sh,
                     float dist, uint64_t seed, const int32_t *pixels, int npx, int threads, int order,
                     int per_sample, float *out, uint64_t *stats)
{
    try {
        std::unique_ptr<Scene> scene = load_scene(scene_text);
        std::atomic<int> next(0);
        std::mutex mu;
        Stats total;
        std::string err;
        auto worker = [&]() {
            Tracer<SampleEngine> tr(*scene, order == 1 ? ORDER_FAST : ORDER_REFERENCE);
            for (uint64_t &c : tl_tex) c = 0;
            try {
                for (;;) {
                    int k = next.fetch_add(1);
                    if (k >= npx)
                        break;
                    int p = pixels ? pixels[k] : k;
                    int px = p % gw, py = p / gw;
                    V3 acc = pixel_sum(spp, order == 1 ? ORDER_FAST : ORDER_REFERENCE, [&](int s) {
                        SampleEngine e(seed, (uint64_t)p, (uint64_t)s);
                        V3 c = tr.sample(px, py, W, H, depth, sw, sh, dist, e);
                        if (per_sample) {
                            float *o = out + ((size_t)k * spp + s) * 3;
                            o[0] = c.x, o[1] = c.y, o[2] = c.z;
                        }
                        return c;
                    });
                    acc = acc / (float)spp;
                    if (!per_sample) {
                        out[3 * (size_t)k + 0] = acc.x;
                        out[3 * (size_t)k + 1] = acc.y;
                        out[3 * (size_t)k + 2] = acc.z;
                    }
                }
            } catch (std::exception &e) {
                std::lock_guard<std::mutex> g(mu);
                err = e.what();
            }
            std::lock_guard<std::mutex> g(mu);
            for (int c = 0; c < TC_N; c++) tr.st.tex[c] = tl_tex[c];
            total.add(tr.st);
        };
        std::vector<std::thread> pool;
        for (int t = 0; t < (threads < 1 ? 1 : threads); t++) pool.emplace_back(worker);
        for (auto &t : pool) t.join();
        if (!err.empty())
            throw std::runtime_error(err);
        if (stats) {
            for (int c = 0; c < TC_N; c++) stats[11 + c] = total.tex[c];
            uint64_t v[11] = {total.queries,          total.sphere_tests,     total.sphere_hits, total.plane_tests,
                              total.merge_steps,      total.shaded,           total.refract_children,
                              total.scatter_children, total.attempts,         total.draws,
                              total.leaf_children};
            memcpy(stats, v, sizeof(v));
        }
        return 0;
    } catch (std::exception &e) {
        g_err = e.what();
        return -1;
    }
}

/* traceRay<T>(ray, it, depth, engine, strength), include/path-trace.h:58-165,
 * for n caller rays (7 floats: origin, direction, strength): per ray the sum of
 * spp samples in `order` (pixel_sum), sample s drawing from the engine keyed
 * (seed, ray_begin + ray index, sample_begin + s), each sample (0 + c) / 1 as a one-sample
 * tracePixel adds it, divided by spp -- what pt_trace_rays computes. */
int oracle_trace_rays(const char *scene_text, const float *rays, int n, int spp, int depth, uint64_t seed,
                      int sample_begin, int64_t ray_begin, int threads, int order, float *out)
{
    try {
        std::unique_ptr<Scene> scene = load_scene(scene_text);
        std::atomic<int> next(0);
        std::mutex mu;
        std::string err;
        auto worker = [&]() {
            Tracer<SampleEngine> tr(*scene, order == 1 ? ORDER_FAST : ORDER_REFERENCE);
            try {
                for (;;) {
                    int k = next.fetch_add(1);
                    if (k >= n)
                        break;
                    const float *r = rays + 7 * (size_t)k;
                    const Ray ray{V3(r[0], r[1], r[2]), V3(r[3], r[4], r[5])};
                    V3 acc = pixel_sum(spp, order == 1 ? ORDER_FAST : ORDER_REFERENCE, [&](int s) {
                        SampleEngine e(seed, (uint64_t)(ray_begin + k), (uint64_t)(sample_begin + s));
                        V3 c = V3(0, 0, 0) + tr.trace(ray, depth, e, r[6]);
                        return c / (float)1;
                    });
                    acc = acc / (float)spp;
                    out[3 * (size_t)k + 0] = acc.x, out[3 * (size_t)k + 1] = acc.y, out[3 * (size_t)k + 2] = acc.z;
                }
            } catch (std::exception &e) {
                std::lock_guard<std::mutex> g(mu);
                err = e.what();
            }
        };
        std::vector<std::thread> pool;
        for (int t = 0; t < (threads < 1 ? 1 : threads); t++) pool.emplace_back(worker);
        for (auto &t : pool) t.join();
        if (!err.empty())
            throw std::runtime_error(err);
        return 0;
    } catch (std::exception &e) {
        g_err = e.what();
        return -1;
    }
}

/* Full root span list per ray; layout as ptref's "spans" mode:
 * int32 count, then count * (t0 n0.xyz m0 t1 n1.xyz m1) with m as int32. */
int oracle_spans(const char *scene_text, const float *rays, int n, char *out, int64_t cap, int64_t *written)
{
    try {
        std::unique_ptr<Scene> scene = load_scene(scene_text);
        Stats st;
        int64_t pos = 0;
        auto put = [&](const void *p, size_t k) {
            if (pos + (int64_t)k > cap)
                throw std::runtime_error("oracle_spans: output buffer too small");
            memcpy(out + pos, p, k);
            pos += k;
        };
        for (int k = 0; k < n; k++) {
            Ray r{V3(rays[6 * k], rays[6 * k + 1], rays[6 * k + 2]), V3(rays[6 * k + 3], rays[6 * k + 4], rays[6 * k + 5])};
            SpanList l;
            scene->root->spans(r, l, st);
            int32_t c = (int32_t)l.v.size();
            put(&c, 4);
            for (const Span &s : l.v) {
                int32_t m0 = s.m0 ? s.m0->id : -1, m1 = s.m1 ? s.m1->id : -1;
                float a[4] = {s.t0, s.n0.x, s.n0.y, s.n0.z}, b[4] = {s.t1, s.n1.x, s.n1.y, s.n1.z};
                put(a, 16);
                put(&m0, 4);
                put(b, 16);
                put(&m1, 4);
            }
        }
        *written = pos;
        return 0;
    } catch (std::exception &e) {
        g_err = e.what();
        return -1;
    }
}

/* Texture::getColor / getFloat of every texture of the scene text (in file
 * order) at n points; layout as ptref's "tex" mode: per texture, per point,
 * r g b value (float32). */
int oracle_tex_eval(const char *scene_text, const float *pts, int n, float *out)
{
    try {
        scenetext::Desc d = scenetext::parse(scene_text);
        std::unique_ptr<Scene> scene = load_scene(scene_text);
        size_t o = 0;
        for (const scenetext::Item &t : d.textures) {
            std::unique_ptr<Tex> tex = make_tex(d, *scene, t.id);
            for (int k = 0; k < n; k++) {
                const V3 p(pts[3 * k], pts[3 * k + 1], pts[3 * k + 2]);
                const V3 c = tex->color(p);
                out[o++] = c.x, out[o++] = c.y, out[o++] = c.z, out[o++] = tex->value(p);
            }
        }
        return 0;
    } catch (std::exception &e) {
        g_err = e.what();
        return -1;
    }
}

/* Vector-math known answers in the exact layout of ptref's "kat" mode, so the
 * two can be compared word for word. */
int oracle_kat(uint32_t *out, int64_t cap, int64_t *written)
{
    std::vector<uint32_t> o;
    auto pf = [&](float f) {
        uint32_t x;
        memcpy(&x, &f, 4);
        o.push_back(x);
    };
    unsigned seeds[3] = {0, 1, 12345};
    for (unsigned s : seeds) {
        LcgEngine e(s);
        for (int k = 0; k < 5; k++) o.push_back(e());
    }
    {
        SampleEngine e(0x5EEDull, 7, 3);
        for (int k = 0; k < 16; k++) o.push_back(e());
    }
    {
        LcgEngine e(0);
        for (int k = 0; k < 4; k++) pf(uniform(e, 0.0f, 1.0f));
        for (int k = 0; k < 4; k++) pf(uniform(e, -1.0f, 1.0f));
    }
    {
        SampleEngine e(0x5EEDull, 1, 1);
        for (int k = 0; k < 64; k++) {
            V3 v;
            do {
                v.x = uniform(e, -1.0f, 1.0f);
                v.y = uniform(e, -1.0f, 1.0f);
                v.z = uniform(e, -1.0f, 1.0f);
            } while (length(v) > 1);
            pf(v.x), pf(v.y), pf(v.z);
        }
    }
    {
        SampleEngine e(0x5EEDull, 2, 2);
        for (int k = 0; k < 256; k++) {
            V3 d, n;
            d.x = uniform(e, -2.0f, 2.0f), d.y = uniform(e, -2.0f, 2.0f), d.z = uniform(e, -2.0f, 2.0f);
            n.x = uniform(e, -2.0f, 2.0f), n.y = uniform(e, -2.0f, 2.0f), n.z = uniform(e, -2.0f, 2.0f);
            float ior = 0.25f + (uniform(e, -2.0f, 2.0f) + 2) * 0.5f;
            if (k % 17 == 0)
                d = V3(0.3f, 0, -1), n = V3(0, 0, 1), ior = 1 / 1.3f;
            V3 r = refract(d, ior, n), rf = reflect(d, n), nn = normalize(d);
            float rs = refract_strength(d, ior, n);
            for (float f : {d.x, d.y, d.z, n.x, n.y, n.z, ior, r.x, r.y, r.z, rs, rf.x, rf.y, rf.z, nn.x, nn.y, nn.z})
                pf(f);
        }
    }
    if ((int64_t)o.size() > cap)
        return -1;
    memcpy(out, o.data(), o.size() * 4);
    *written = (int64_t)o.size();
    return 0;
}

} // extern "C"
