/* internal.h -- host-side data model of libpt.so (not part of the C ABI). */
#ifndef PT_INTERNAL_H
#define PT_INTERNAL_H

#include <cstdint>
#include <map>
#include <memory>
#include <mutex>
#include <stdexcept>
#include <string>
#include <vector>

#include "../../include/pt/pt.h"

namespace pt
{

/* An error carrying a C-ABI status code; caught at every extern "C" boundary. */
struct Error : std::runtime_error
{
    int code;
    Error(int c, const std::string &m) : std::runtime_error(m), code(c) {}
};

void set_error(const std::string &msg);

/* Host copies of the reference scene graph, one record per constructor call. */
struct ImageRec
{
    int w = 0, h = 0;
    std::vector<float> rgba; /* row 0 = top */
};

enum class TexKind { Color, Image, ImageAlpha, Skybox, SkyboxAlpha, Multiply, Log, MirrorBall, Spherical, Xform, Coord, User };

struct TexRec
{
    TexKind kind;
    float f[12] = {0};
    int child = -1;   /* inner texture */
    int img[6] = {-1, -1, -1, -1, -1, -1};
    /* User (pt_tex_device): the caller's device bodies and parameters */
    std::string color_body, value_body;
    std::vector<float> params;
};

struct MatRec
{
    int reflect, scatter, emissive, transmit, trc;
    float ior;
};

enum class ObjKind { Sphere, Plane, Union, Intersection, Difference, Xform, User };

struct ObjRec
{
    ObjKind kind;
    float f[12] = {0}; /* sphere: c, r; plane: n, d; xform: m */
    int mat = -1;
    int a = -1, b = -1; /* children */
    /* User (pt_object_device): the caller's device bodies and parameters */
    std::string span_body, normal_body;
    std::vector<float> params;
};

struct DeviceState; /* runtime.cpp */
struct Generated;

struct SceneImpl
{
    std::vector<ImageRec> images;
    std::vector<TexRec> textures;
    std::vector<MatRec> materials;
    std::vector<ObjRec> objects;
    int root = -1;
    int default_tex[2] = {-1, -1}; /* lazily created ColorTexture(0), ColorTexture(1) */
    int wg_per_cu = 0;             /* resident workgroups per CU the kernel is built for (0 = auto) */
    int fast_spine = 0;            /* spine queries try all spans + the fast checks first */
    int lane_walk = 0;             /* register frames of the per-lane scatter-free tree walk (0 = off) */
    int lane_scatter = 0;          /* per-lane walk of whole trees, scatter loops included */
    int split = 1;                 /* lane-walk scenes: light kernel first (launch-time only) */
    std::map<int, std::unique_ptr<DeviceState>> devices;
    std::shared_ptr<struct QueryCache> qcache; /* loaded query modules (runtime.cpp) */
    std::string last_key;
    /* generated render modules by a fingerprint of everything generate() reads
     * (runtime.cpp generated(): per-call callers skip the ~200 KB source text) */
    std::map<uint64_t, std::shared_ptr<const Generated>> gen_cache;
    void clear()
    {
        images.clear(), textures.clear(), materials.clear(), objects.clear();
        gen_cache.clear();
        qcache.reset(); /* its modules hold copies of the old images */
        root = -1;
        default_tex[0] = default_tex[1] = -1;
    }
};

/* Generated device module for one (scene, depth). */
struct Generated
{
    std::string source;         /* full hiprtc translation unit                      */
    std::string key;            /* content hash of the source (code_object_key adds options + compiler) */
    std::vector<float> params;  /* scene parameter block P                           */
    std::vector<int> image_ids; /* slot -> scene image index                          */
    std::vector<int> mat_ids;   /* compact material index -> scene material index     */
    int maxd = 0;
    int n_prims = 0, n_spheres = 0, n_planes = 0, n_mats = 0;
    std::vector<std::string> options; /* per-scene compiler options (part of the code-object key) */
};

/* rays: the module of pt_trace_rays (PT_RAYS), whose items are caller rays */
Generated generate(const SceneImpl &s, int depth, bool rays = false);
/* Query module for the boundary's query virtuals: pt_query_spans over object
 * `obj` (if >= 0) and pt_tex_eval of texture `tex` (if >= 0). */
Generated generate_query(const SceneImpl &s, int obj, int tex);
/* Returns the gfx950 code object for g (from the cache or compiled now). */
const std::vector<char> &code_object(const Generated &g);
/* The code object's cache key: source + compiler options + hiprtc version
 * (the _jit_cache file name; what a profile is bound to). */
std::string code_object_key(const Generated &g);

/* Matrix helpers (reference include/transform.h arithmetic). */
void mat_inverse(const float *m, float *out); /* throws Error(PT_ERR_MATH) */
void mat_concat(const float *a, const float *b, float *out);
void mat_rotate(const float *axis, double angle, float *out);

/* Image I/O (reference src/image.cpp). */
ImageRec read_hdr(const std::string &path);
ImageRec read_png(const std::string &path);
ImageRec read_image(const std::string &path);
void write_hdr(const std::string &path, const float *rgb, int w, int h);
void write_bmp(const std::string &path, const float *rgb, int w, int h, int count);

std::string device_library_source(); /* embedded pt_device.h */
std::string device_user_object_source(); /* embedded pt_user_object.h (scenes with user objects) */

} // namespace pt

#endif
