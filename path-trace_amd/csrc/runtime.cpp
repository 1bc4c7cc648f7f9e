/*
 * runtime.cpp -- libpt.so: the C-ABI boundary (include/pt/pt.h).
 *
 * Holds the host copy of the scene graph built through the reference-shaped
 * constructors, flattens it into a device module (codegen.cpp), gets the
 * gfx950 code object (jit.cpp), and drives the megakernel:
 *
 *   items = (pixel slot, sample) pairs; a persistent grid of waves pulls
 *   chunks of up to 32 items from a counter (pt_render_fast / _strict),
 *   slot-major for large launches, sample-major for launches of <= 64 samples
 *   per slot.  Reference order stages each sample's radiance and pt_reduce
 *   sums a pixel's samples in sample order, exactly tracePixel's loop; the
 *   fast order stages one pairwise partial per 32-sample block (whole
 *   blocks per chunk) or per-sample values, and pt_reduce adds the blocks in
 *   order.  Large frames run in sample passes bounded by max_buffer_bytes,
 *   the running per-pixel sums carried between passes.
 *
 * This replaces RenderBlock::calcPixelColor's per-pixel tracePixel calls
 * (reference src/test.cpp:441-465); the block farm / thread pool around it
 * (src/test.cpp:147-518) becomes the hardware dispatcher plus, across GPUs,
 * one process per device (bench.py / pathtrace.dist).
 */
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <climits>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <functional>
#include <map>
#include <sstream>

#include "../../include/pt/pt_engine.h"
#include "internal.h"

struct pt_scene
{
    pt::SceneImpl impl;
};

namespace pt
{

thread_local std::string g_error;
void set_error(const std::string &msg) { g_error = msg; }

/* Host-clock phases of this thread's last pt_render (pt_call_profile). */
thread_local double g_prof[PT_PROF_N];
double now_us()
{
    return (double)std::chrono::duration_cast<std::chrono::nanoseconds>(
               std::chrono::steady_clock::now().time_since_epoch())
               .count() /
           1e3;
}

#define HIPCHECK(x)                                                                                  \
    do {                                                                                             \
        hipError_t e_ = (x);                                                                         \
        if (e_ != hipSuccess)                                                                        \
            throw Error(PT_ERR_DEVICE, std::string(#x) + ": " + hipGetErrorString(e_));              \
    } while (0)

struct PtImageDev
{
    const void *data;
    uint32_t w, h;
};

struct PtLaunchHost /* must match ptd::PtLaunch */
{
    uint64_t seed;
    long long n_items;
    long long chunk0;
    int W, H;
    float sw, sh, dist;
    int depth;
    int nsamp;
    int s0;
    int gw, chunk;
    int sample_major;
    int block_sums;
    long long perm;
    const float *rays;
    long long ray0;
    int grab;
    const unsigned *list;
    unsigned *bail;
};

template <class T>
struct DevBuf
{
    T *p = nullptr;
    size_t n = 0;
    void ensure(size_t count)
    {
        if (count <= n)
            return;
        release();
        HIPCHECK(hipMalloc((void **)&p, count * sizeof(T)));
        n = count;
    }
    void release()
    {
        if (p)
            (void)hipFree(p);
        p = nullptr;
        n = 0;
    }
};

/* Page-locked host staging (grow-only): transfers from and to it are true
 * DMA, with no driver-side staging copy (pt_render's small per-call transfers) */
template <class T>
struct PinBuf
{
    T *p = nullptr;
    size_t n = 0;
    void ensure(size_t count)
    {
        if (count <= n)
            return;
        release();
        HIPCHECK(hipHostMalloc((void **)&p, count * sizeof(T), hipHostMallocDefault));
        n = count;
    }
    void release()
    {
        if (p)
            (void)hipHostFree(p);
        p = nullptr;
        n = 0;
    }
};

/* The HIP events and sample count of one render whose timings are not read yet */
struct PendingRender
{
    std::vector<hipEvent_t> evs;
    std::vector<std::pair<int, int>> spans, rspans; /* (start, end) event of each render / reduce launch */
    uint64_t samples = 0;
    int n_spheres = 0, n_planes = 0;
};

struct DeviceState
{
    int device = 0;
    std::string key;
    hipModule_t mod = nullptr;
    hipFunction_t fast = nullptr, strict = nullptr, reduce = nullptr;
    hipFunction_t light = nullptr; /* lane-walk modules: the split launch's light kernel */
    int wpw = 1; /* waves (chunks of 64 items) per workgroup, from the kernel's launch bounds */
    int resident_blocks = 0; /* persistent grid size: resident workgroups per CU x CUs */
    int light_blocks = 0;    /* the same for the light kernel */
    DevBuf<unsigned> bail;   /* the chunks the light kernel leaves to the full one */
    std::vector<float> params;
    DevBuf<float> P;
    DevBuf<PtImageDev> imgs;
    std::vector<DevBuf<float>> img_data;
    std::vector<int> img_ids;
    DevBuf<uint64_t> jump;
    DevBuf<float> stage, accum, fb;
    DevBuf<float> out; /* pt_render's output (grow-only: no allocation per call) */
    PinBuf<int> hpix;  /* pt_render's pixel list and result, staged in pinned memory */
    PinBuf<float> hout;
    DevBuf<int> pixels;
    DevBuf<uint64_t> stats;
    std::vector<PendingRender> pending; /* deferred timings (pt_render_device_timed) */
    ~DeviceState()
    {
        int prev = 0;
        if (hipGetDevice(&prev) == hipSuccess && hipSetDevice(device) == hipSuccess) {
            for (auto &pr : pending)
                for (auto e : pr.evs) (void)hipEventDestroy(e);
            P.release(), imgs.release(), jump.release(), stage.release(), accum.release(), fb.release();
            out.release(), hpix.release(), hout.release();
            pixels.release(), stats.release();
            for (auto &b : img_data) b.release();
            if (mod)
                (void)hipModuleUnload(mod);
            (void)hipSetDevice(prev);
        }
    }
};

/* ------------------------------------------------------------ matrices -- */
/* transform.h:342-383 */
void mat_inverse(const float *m, float *out)
{
    const float x00 = m[0], x10 = m[1], x20 = m[2], x30 = m[3], x01 = m[4], x11 = m[5], x21 = m[6], x31 = m[7],
                x02 = m[8], x12 = m[9], x22 = m[10], x32 = m[11];
    float det = x00 * (x11 * x22 - x12 * x21) + x10 * (x02 * x21 - x01 * x22) + x20 * (x01 * x12 - x02 * x11);
    if (det == 0.0f)
        throw Error(PT_ERR_MATH, "can't invert singular matrix");
    float f = 1.0f / det;
    out[0] = (x11 * x22 - x12 * x21) * f;
    out[1] = (x12 * x20 - x10 * x22) * f;
    out[2] = (x10 * x21 - x11 * x20) * f;
    out[3] = (-x10 * x21 * x32 + x11 * x20 * x32 + x10 * x22 * x31 - x12 * x20 * x31 - x11 * x22 * x30 +
              x12 * x21 * x30) *
             f;
    out[4] = (x02 * x21 - x01 * x22) * f;
    out[5] = (x00 * x22 - x02 * x20) * f;
    out[6] = (x01 * x20 - x00 * x21) * f;
    out[7] = (x00 * x21 * x32 - x01 * x20 * x32 - x00 * x22 * x31 + x02 * x20 * x31 + x01 * x22 * x30 -
              x02 * x21 * x30) *
             f;
    out[8] = (x01 * x12 - x02 * x11) * f;
    out[9] = (x02 * x10 - x00 * x12) * f;
    out[10] = (x00 * x11 - x01 * x10) * f;
    out[11] = (-x00 * x11 * x32 + x01 * x10 * x32 + x00 * x12 * x31 - x02 * x10 * x31 - x01 * x12 * x30 +
               x02 * x11 * x30) *
              f;
}

/* Matrix::concat, transform.h:391-406: this->concat(rt) = "apply this, then rt" */
void mat_concat(const float *a, const float *b, float *out)
{
    const float t00 = a[0], t10 = a[1], t20 = a[2], t30 = a[3], t01 = a[4], t11 = a[5], t21 = a[6], t31 = a[7],
                t02 = a[8], t12 = a[9], t22 = a[10], t32 = a[11];
    const float r00 = b[0], r10 = b[1], r20 = b[2], r30 = b[3], r01 = b[4], r11 = b[5], r21 = b[6], r31 = b[7],
                r02 = b[8], r12 = b[9], r22 = b[10], r32 = b[11];
    out[0] = t00 * r00 + t01 * r10 + t02 * r20;
    out[1] = t10 * r00 + t11 * r10 + t12 * r20;
    out[2] = t20 * r00 + t21 * r10 + t22 * r20;
    out[3] = t30 * r00 + t31 * r10 + t32 * r20 + r30;
    out[4] = t00 * r01 + t01 * r11 + t02 * r21;
    out[5] = t10 * r01 + t11 * r11 + t12 * r21;
    out[6] = t20 * r01 + t21 * r11 + t22 * r21;
    out[7] = t30 * r01 + t31 * r11 + t32 * r21 + r31;
    out[8] = t00 * r02 + t01 * r12 + t02 * r22;
    out[9] = t10 * r02 + t11 * r12 + t12 * r22;
    out[10] = t20 * r02 + t21 * r12 + t22 * r22;
    out[11] = t30 * r02 + t31 * r12 + t32 * r22 + r32;
}

/* Matrix::rotate, transform.h:207-225 (cos/sin of a double angle, float math) */
void mat_rotate(const float *axis, double angle, float *out)
{
    float ax = axis[0], ay = axis[1], az = axis[2];
    float m = std::sqrt((ax * ax + ay * ay) + az * az);
    if (m == 0)
        m = 1;
    ax /= m, ay /= m, az /= m;
    float c = (float)std::cos(angle), s = (float)std::sin(angle), v = 1 - c;
    float xx = ax * ax, xy = ax * ay, xz = ax * az, yy = ay * ay, yz = ay * az, zz = az * az;
    float r[12] = {xx + (1 - xx) * c, xy * v - az * s, xz * v + ay * s, 0, xy * v + az * s, yy + (1 - yy) * c,
                   yz * v - ax * s,   0,               xz * v - ay * s, yz * v + ax * s, zz + (1 - zz) * c, 0};
    memcpy(out, r, sizeof r);
}

/* -------------------------------------------------------------- helpers -- */
namespace
{

SceneImpl &S(pt_scene *s)
{
    if (!s)
        throw Error(PT_ERR_ARG, "null scene");
    return s->impl;
}

void check_img(const SceneImpl &s, int id)
{
    if (id < 0 || id >= (int)s.images.size())
        throw Error(PT_ERR_ARG, "bad image id " + std::to_string(id));
}
void check_tex(const SceneImpl &s, int id)
{
    if (id < 0 || id >= (int)s.textures.size())
        throw Error(PT_ERR_ARG, "bad texture id " + std::to_string(id));
}
void check_mat(const SceneImpl &s, int id)
{
    if (id < 0 || id >= (int)s.materials.size())
        throw Error(PT_ERR_ARG, "bad material id " + std::to_string(id));
}
void check_obj(const SceneImpl &s, int id)
{
    if (id < 0 || id >= (int)s.objects.size())
        throw Error(PT_ERR_ARG, "bad object id " + std::to_string(id));
}

int add_tex(SceneImpl &s, const TexRec &t)
{
    s.textures.push_back(t);
    return (int)s.textures.size() - 1;
}

int default_tex(SceneImpl &s, int which) /* ColorTexture(0) / ColorTexture(1) */
{
    TexRec t;
    t.kind = TexKind::Color;
    t.f[0] = t.f[1] = t.f[2] = (float)which;
    return add_tex(s, t);
}

template <class F>
int guard(F f)
{
    try {
        return f();
    } catch (Error &e) {
        set_error(e.what());
        return e.code;
    } catch (std::exception &e) {
        set_error(e.what());
        return PT_ERR_ARG;
    }
}

std::string trim(const std::string &s)
{
    size_t a = s.find_first_not_of(" \t\r"), b = s.find_last_not_of(" \t\r");
    return a == std::string::npos ? "" : s.substr(a, b - a + 1);
}

float tof(const std::string &t)
{
    char *end = nullptr;
    float v = strtof(t.c_str(), &end);
    if (end == t.c_str() || *end)
        throw Error(PT_ERR_ARG, "bad float '" + t + "'");
    return v;
}

int toi(const std::string &t)
{
    char *end = nullptr;
    long v = strtol(t.c_str(), &end, 10);
    if (end == t.c_str() || *end)
        throw Error(PT_ERR_ARG, "bad int '" + t + "'");
    return (int)v;
}

/* Loads the plain-text scene format into s (ids are renumbered). */
void load_text(SceneImpl &s, const std::string &text)
{
    s.clear();
    std::map<int, int> img, tex, mat, obj;
    std::istringstream in(text);
    std::string line;
    int root = -1;
    auto need = [](const std::vector<std::string> &t, size_t n) {
        if (t.size() != n)
            throw Error(PT_ERR_ARG, "scene text: wrong operand count near '" + (t.empty() ? "" : t[0]) + "'");
    };
    auto look = [](std::map<int, int> &m, int id, const char *what) {
        auto it = m.find(id);
        if (it == m.end())
            throw Error(PT_ERR_ARG, std::string("scene text: unknown ") + what + " " + std::to_string(id));
        return it->second;
    };
    while (std::getline(in, line)) {
        line = trim(line);
        if (line.empty() || line[0] == '#')
            continue;
        std::istringstream ls(line);
        std::vector<std::string> t;
        std::string w;
        while (ls >> w) t.push_back(w);
        const std::string &k = t[0];
        if (k == "root") {
            need(t, 2);
            root = look(obj, toi(t[1]), "object");
            continue;
        }
        if (t.size() < 3)
            throw Error(PT_ERR_ARG, "scene text: short line");
        int id = toi(t[1]);
        const std::string &ty = t[2];
        if (k == "image") {
            if (ty == "hdr") {
                need(t, 4);
                s.images.push_back(read_hdr(t[3]));
            } else if (ty == "png") {
                need(t, 4);
                s.images.push_back(read_png(t[3]));
            } else if (ty == "raw") {
                need(t, 6);
                ImageRec r;
                r.w = toi(t[3]), r.h = toi(t[4]);
                std::ifstream f(t[5], std::ios::binary);
                if (!f)
                    throw Error(PT_ERR_IO, "can't open " + t[5]);
                r.rgba.resize((size_t)4 * r.w * r.h);
                f.read((char *)r.rgba.data(), (std::streamsize)(r.rgba.size() * 4));
                if (!f)
                    throw Error(PT_ERR_IO, "short raw image " + t[5]);
                s.images.push_back(std::move(r));
            } else
                throw Error(PT_ERR_ARG, "scene text: image kind " + ty);
            img[id] = (int)s.images.size() - 1;
        } else if (k == "tex") {
            TexRec r;
            if (ty == "color") {
                need(t, 6);
                r.kind = TexKind::Color;
                for (int j = 0; j < 3; j++) r.f[j] = tof(t[3 + j]);
            } else if (ty == "coord") {
                need(t, 3);
                r.kind = TexKind::Coord;
            } else if (ty == "image" || ty == "image_alpha") {
                need(t, 4);
                r.kind = ty == "image" ? TexKind::Image : TexKind::ImageAlpha;
                r.img[0] = look(img, toi(t[3]), "image");
            } else if (ty == "skybox" || ty == "skybox_alpha") {
                need(t, 9);
                r.kind = ty == "skybox" ? TexKind::Skybox : TexKind::SkyboxAlpha;
                for (int j = 0; j < 6; j++) r.img[j] = look(img, toi(t[3 + j]), "image");
            } else if (ty == "multiply") {
                need(t, 7);
                r.kind = TexKind::Multiply;
                for (int j = 0; j < 3; j++) r.f[j] = tof(t[3 + j]);
                r.child = look(tex, toi(t[6]), "texture");
            } else if (ty == "log" || ty == "mirrorball" || ty == "spherical") {
                need(t, 4);
                r.kind = ty == "log" ? TexKind::Log : ty == "mirrorball" ? TexKind::MirrorBall : TexKind::Spherical;
                r.child = look(tex, toi(t[3]), "texture");
            } else if (ty == "xform") {
                need(t, 16);
                r.kind = TexKind::Xform;
                for (int j = 0; j < 12; j++) r.f[j] = tof(t[3 + j]);
                r.child = look(tex, toi(t[15]), "texture");
            } else
                throw Error(PT_ERR_ARG, "scene text: texture kind " + ty);
            tex[id] = add_tex(s, r);
        } else if (k == "mat") {
            need(t, 8);
            MatRec m;
            m.reflect = look(tex, toi(t[2]), "texture");
            m.scatter = look(tex, toi(t[3]), "texture");
            m.emissive = look(tex, toi(t[4]), "texture");
            m.transmit = look(tex, toi(t[5]), "texture");
            m.ior = tof(t[6]);
            m.trc = look(tex, toi(t[7]), "texture");
            s.materials.push_back(m);
            mat[id] = (int)s.materials.size() - 1;
        } else if (k == "obj") {
            ObjRec o;
            if (ty == "sphere" || ty == "plane") {
                need(t, 8);
                o.kind = ty == "sphere" ? ObjKind::Sphere : ObjKind::Plane;
                for (int j = 0; j < 4; j++) o.f[j] = tof(t[3 + j]);
                o.mat = look(mat, toi(t[7]), "material");
            } else if (ty == "union" || ty == "intersection" || ty == "difference") {
                need(t, 5);
                o.kind = ty == "union" ? ObjKind::Union : ty == "intersection" ? ObjKind::Intersection
                                                                                : ObjKind::Difference;
                o.a = look(obj, toi(t[3]), "object");
                o.b = look(obj, toi(t[4]), "object");
            } else if (ty == "xform") {
                need(t, 16);
                o.kind = ObjKind::Xform;
                for (int j = 0; j < 12; j++) o.f[j] = tof(t[3 + j]);
                o.a = look(obj, toi(t[15]), "object");
            } else
                throw Error(PT_ERR_ARG, "scene text: object kind " + ty);
            s.objects.push_back(o);
            obj[id] = (int)s.objects.size() - 1;
        } else
            throw Error(PT_ERR_ARG, "scene text: unknown line kind " + k);
    }
    if (root < 0)
        throw Error(PT_ERR_ARG, "scene text: no root");
    s.root = root;
}

/* jump table (A_{3m}, G_{3m}), m = 0..1024 (PT_KATT <= 16), of state_{n+3m} = A*state_n + G*inc
 * (PT_JUMP_ENTRIES of the device code: up to 16 x 64 attempts per round) */
std::vector<uint64_t> jump_table()
{
    constexpr uint32_t kEntries = 1025;
    std::vector<uint64_t> t(2 * kEntries);
    for (uint32_t m = 0; m < kEntries; m++) pt_lcg_jump_coeffs(3 * m, &t[2 * m], &t[2 * m + 1]);
    return t;
}

/* A scene's state on one device: the render module, or (rays) the ray-list
 * module of pt_trace_rays, each with its own buffers so that alternating calls
 * reload nothing. */
constexpr int kRaysState = 1 << 16;
DeviceState &device_state(SceneImpl &s, int device, const Generated &g, bool rays = false)
{
    HIPCHECK(hipSetDevice(device));
    std::unique_ptr<DeviceState> &ds = s.devices[device | (rays ? kRaysState : 0)];
    if (!ds) {
        ds.reset(new DeviceState);
        ds->device = device;
        std::vector<uint64_t> jt = jump_table();
        ds->jump.ensure(jt.size());
        HIPCHECK(hipMemcpy(ds->jump.p, jt.data(), jt.size() * 8, hipMemcpyHostToDevice));
        ds->stats.ensure(40);
    }
    if (ds->key != g.key) {
        const std::vector<char> &code = code_object(g);
        if (ds->mod)
            HIPCHECK(hipModuleUnload(ds->mod));
        ds->mod = nullptr;
        HIPCHECK(hipModuleLoadData(&ds->mod, code.data()));
        HIPCHECK(hipModuleGetFunction(&ds->fast, ds->mod, "pt_render_fast"));
        HIPCHECK(hipModuleGetFunction(&ds->strict, ds->mod, "pt_render_strict"));
        HIPCHECK(hipModuleGetFunction(&ds->reduce, ds->mod, "pt_reduce"));
        int mt = 0;
        HIPCHECK(hipFuncGetAttribute(&mt, HIP_FUNC_ATTRIBUTE_MAX_THREADS_PER_BLOCK, ds->fast));
        if (mt < 64 || mt % 64)
            throw Error(PT_ERR_DEVICE, "unexpected megakernel block size " + std::to_string(mt));
        ds->wpw = mt / 64;
        int per_cu = 0, cus = 0;
        HIPCHECK(hipModuleOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, ds->fast, mt, 0));
        HIPCHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device));
        ds->resident_blocks = std::max(1, per_cu) * std::max(1, cus);
        /* lane-walk modules define pt_render_light (pt_device.h PT_DEFINE_LIGHT) */
        ds->light = nullptr;
        ds->light_blocks = 0;
        if (hipModuleGetFunction(&ds->light, ds->mod, "pt_render_light") != hipSuccess) {
            (void)hipGetLastError();
            ds->light = nullptr;
        } else {
            int lt = 0;
            HIPCHECK(hipFuncGetAttribute(&lt, HIP_FUNC_ATTRIBUTE_MAX_THREADS_PER_BLOCK, ds->light));
            if (lt != mt)
                throw Error(PT_ERR_DEVICE, "light kernel block size differs from the megakernel's");
            HIPCHECK(hipModuleOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, ds->light, mt, 0));
            ds->light_blocks = std::max(1, per_cu) * std::max(1, cus);
        }
        ds->key = g.key;
    }
    if (ds->params != g.params) {
        ds->P.ensure(g.params.size());
        HIPCHECK(hipMemcpy(ds->P.p, g.params.data(), g.params.size() * 4, hipMemcpyHostToDevice));
        ds->params = g.params;
    }
    if (ds->img_ids != g.image_ids) {
        for (auto &b : ds->img_data) b.release();
        ds->img_data.clear();
        ds->img_data.resize(g.image_ids.size());
        std::vector<PtImageDev> desc(g.image_ids.size() + 1);
        for (size_t k = 0; k < g.image_ids.size(); k++) {
            const ImageRec &im = s.images.at(g.image_ids[k]);
            ds->img_data[k].ensure(im.rgba.size());
            HIPCHECK(hipMemcpy(ds->img_data[k].p, im.rgba.data(), im.rgba.size() * 4, hipMemcpyHostToDevice));
            desc[k].data = ds->img_data[k].p;
            desc[k].w = (uint32_t)im.w;
            desc[k].h = (uint32_t)im.h;
        }
        ds->imgs.ensure(desc.size());
        HIPCHECK(hipMemcpy(ds->imgs.p, desc.data(), desc.size() * sizeof(PtImageDev), hipMemcpyHostToDevice));
        ds->img_ids = g.image_ids;
    }
    return *ds;
}

void validate(const pt_render_params *p)
{
    if (!p)
        throw Error(PT_ERR_ARG, "null params");
    if (p->width <= 0 || p->height <= 0 || p->spp <= 0)
        throw Error(PT_ERR_ARG, "width, height and spp must be positive");
    if ((int64_t)p->width * p->height >= (1ll << 31))
        throw Error(PT_ERR_ARG, "frame too large");
    if (p->spp >= (1 << 20))
        throw Error(PT_ERR_ARG, "spp must be < 2^20 (engine key layout)");
    if (p->sample_begin < 0 || (int64_t)p->sample_begin + p->spp > (1 << 20))
        throw Error(PT_ERR_ARG, "samples must lie in [0, 2^20) (engine key layout)");
    if (p->depth < 0 || p->depth > 64)
        throw Error(PT_ERR_ARG, "depth must be in [0, 64]");
    if (p->order != PT_ORDER_FAST && p->order != PT_ORDER_REFERENCE)
        throw Error(PT_ERR_ARG, "bad order");
    if (p->grid_width != 0 && p->grid_width < p->width)
        throw Error(PT_ERR_ARG, "grid_width must be 0 or >= width");
    if (p->pixels) {
        const int64_t limit = p->grid_width ? (int64_t)INT32_MAX : (int64_t)p->width * p->height;
        for (int64_t k = 0; k < p->npixels; k++)
            if (p->pixels[k] < 0 || p->pixels[k] >= limit)
                throw Error(PT_ERR_ARG, "pixel index out of range");
    }
}

/* frame-buffer floats a render with p addresses */
size_t frame_floats(const pt_render_params *p)
{
    size_t n = (size_t)p->width * p->height;
    if (p->pixels)
        for (int64_t k = 0; k < p->npixels; k++) n = std::max(n, (size_t)p->pixels[k] + 1);
    return 3 * n;
}

/* The fast order sums a pixel's samples in blocks of 32 (pt_device.h
 * pt_reduce); a slot-major launch of whole blocks stages one partial per
 * block instead of one value per sample (32x less: C4 3.2 GB, C5 25 GB in one
 * pass). */
bool block_staging(const pt_render_params *p)
{
    static const bool off = [] {
        const char *env = getenv("PT_BLOCK_SUMS"); /* experiment hook: 0 = per-sample staging only */
        if (!env || !*env)
            return false;
        fprintf(stderr, "pt: experiment hook PT_BLOCK_SUMS=%s active\n", env);
        return atoi(env) == 0;
    }();
    return !off && p->order == PT_ORDER_FAST && p->spp > 64 && p->spp % 32 == 0;
}

long long pass_samples(const pt_render_params *p, long long npix)
{
    int64_t budget = p->max_buffer_bytes > 0 ? p->max_buffer_bytes : (8ll << 30);
    long long per_pass = budget / (12ll * npix) * (block_staging(p) ? 32 : 1);
    per_pass = per_pass / 64 * 64;
    if (per_pass < 64)
        per_pass = 64;
    if (per_pass > p->spp)
        per_pass = p->spp;
    return per_pass;
}

/* Multiplier of the sample-major slot permutation (pt_device.h item_slot): a
 * prime near nslots / phi that does not divide nslots, so consecutive slots
 * of a chunk land ~0.38 of the list apart; 0 (identity) below 128 slots or
 * with PT_SAMPLE_PERM=0 (experiment hook). */
long long slot_permutation(long long nslots)
{
    static const bool on = [] {
        const char *env = getenv("PT_SAMPLE_PERM");
        if (env && *env == '0') {
            fprintf(stderr, "pt: experiment hook PT_SAMPLE_PERM=0 active\n");
            return false;
        }
        return true;
    }();
    if (!on || nslots < 128)
        return 0;
    auto prime = [](long long v) {
        if (v < 2)
            return false;
        for (long long d = 2; d * d <= v; d++)
            if (v % d == 0)
                return false;
        return true;
    };
    for (long long m = (long long)((double)nslots * 0.6180339887) | 1; m > 2; m -= 2)
        if (prime(m) && nslots % m != 0)
            return m;
    return 0;
}

/* split launches of lane-walk modules (pt_render_light + pt_render_fast);
 * PT_SPLIT=0 is an experiment hook: every chunk through the full kernel */
bool split_launches()
{
    static const bool on = [] {
        const char *env = getenv("PT_SPLIT");
        if (!env || !*env)
            return true;
        fprintf(stderr, "pt: experiment hook PT_SPLIT=%s active\n", env);
        return atoi(env) != 0;
    }();
    return on;
}

/* Chunks a wave takes per work-queue atomic while its chunks are cheap and
 * plenty are left (pt_device.h render_chunk): 8 in lane-walk scenes, whose
 * chunks are uniformly cheap and whose launches the single counter's atomic
 * rate bounds (C5 5 296 -> 8 112 Msamples/s), 1 elsewhere (C3: -0.45 % with
 * runs).  PT_GRAB=n is an experiment hook. */
int grab_chunks(const SceneImpl &s)
{
    static const int env_g = [] {
        const char *env = getenv("PT_GRAB");
        if (!env || !*env)
            return 0;
        fprintf(stderr, "pt: experiment hook PT_GRAB=%s active\n", env);
        return std::max(1, std::min(64, atoi(env)));
    }();
    if (env_g)
        return env_g;
    return (s.lane_walk > 0 || s.lane_scatter) ? 8 : 1;
}

/* Stage floats for the largest launch of a render: block partials for
 * slot-major whole-block launches, else one value per sample -- launches of
 * <= 64 samples per slot (sample-major) and small launches whose chunks fall
 * below 32 items (at most 4 * 32 items per resident wave). */
size_t stage_floats(const pt_render_params *p, long long npix, long long per_pass)
{
    if (!block_staging(p))
        return (size_t)(npix * per_pass * 3);
    size_t n = (size_t)(npix * (per_pass / 32) * 3);
    n = std::max(n, (size_t)(npix * std::min<long long>(64, p->spp) * 3));
    n = std::max(n, (size_t)(4ll * 64 * 16384 * 3)); /* a small launch: < 4 chunks of 64 per wave, <= 16384 waves */
    return std::min(n, (size_t)(npix * per_pass * 3));
}

/* generate() is a pure function of the scene records, the depth, the module
 * kind and the experiment hooks it reads; its text (the ~200 KB device library
 * plus the scene's types) and the FNV key over it cost about 0.1 ms, which a
 * caller tracing pixel by pixel (src/test.cpp:450) would pay per call.  A
 * scene keeps what it generated under a fingerprint of those inputs. */
struct Fnv
{
    uint64_t h = 0xcbf29ce484222325ull;
    void bytes(const void *p, size_t n)
    {
        const unsigned char *b = (const unsigned char *)p;
        for (size_t k = 0; k < n; k++) h = (h ^ b[k]) * 0x100000001b3ull;
    }
    template <class T>
    void add(const T &v)
    {
        bytes(&v, sizeof v);
    }
    void str(const char *v)
    {
        const size_t n = v ? strlen(v) : (size_t)-1;
        add(n);
        if (v)
            bytes(v, n);
    }
};
std::shared_ptr<const Generated> generated(SceneImpl &s, int depth, bool rays)
{
    if (const char *hdr = getenv("PT_DEVICE_HEADER")) /* experiment hook: the file may change under us */
        if (*hdr)
            return std::make_shared<const Generated>(generate(s, depth, rays));
    Fnv f;
    for (const ObjRec &o : s.objects) {
        f.add(o.kind), f.add(o.mat), f.add(o.a), f.add(o.b);
        f.bytes(o.f, sizeof o.f);
        f.str(o.span_body.c_str()), f.str(o.normal_body.c_str());
        f.add(o.params.size());
        if (!o.params.empty())
            f.bytes(o.params.data(), o.params.size() * sizeof(float));
    }
    f.add(s.objects.size());
    for (const MatRec &m : s.materials) {
        f.add(m.reflect), f.add(m.scatter), f.add(m.emissive), f.add(m.transmit), f.add(m.trc), f.add(m.ior);
    }
    f.add(s.materials.size());
    for (const TexRec &t : s.textures) {
        f.add(t.kind), f.add(t.child);
        f.bytes(t.f, sizeof t.f), f.bytes(t.img, sizeof t.img);
        f.str(t.color_body.c_str()), f.str(t.value_body.c_str());
        f.add(t.params.size());
        if (!t.params.empty())
            f.bytes(t.params.data(), t.params.size() * sizeof(float));
    }
    f.add(s.textures.size());
    for (const ImageRec &im : s.images) /* images are immutable once created */
        f.add(im.w), f.add(im.h);
    f.add(s.images.size());
    f.add(s.root), f.add(s.default_tex[0]), f.add(s.default_tex[1]);
    f.add(s.wg_per_cu), f.add(s.fast_spine), f.add(s.lane_walk), f.add(s.lane_scatter);
    f.add(depth), f.add(rays);
    f.str(getenv("PT_DEVICE_DEFINES")), f.str(getenv("PT_JIT_OPTIONS"));
    auto it = s.gen_cache.find(f.h);
    if (it != s.gen_cache.end())
        return it->second;
    if (s.gen_cache.size() >= 16)
        s.gen_cache.clear();
    auto g = std::make_shared<const Generated>(generate(s, depth, rays));
    s.gen_cache[f.h] = g;
    return g;
}

/* Module, parameters and every device buffer a render with p needs. */
DeviceState &prepare(SceneImpl &s, const pt_render_params *p, std::shared_ptr<const Generated> &gp,
                     bool rays = false)
{
    validate(p);
    gp = generated(s, p->depth, rays);
    const Generated &g = *gp;
    s.last_key = g.key;
    DeviceState &ds = device_state(s, p->device, g, rays);
    const long long npix = p->pixels ? (long long)p->npixels : (long long)p->width * p->height;
    if (npix > 0) {
        long long per_pass = pass_samples(p, npix);
        ds.stage.ensure(stage_floats(p, npix, per_pass));
        if (p->spp > per_pass)
            ds.accum.ensure((size_t)npix * 3);
        if (p->pixels)
            ds.pixels.ensure((size_t)npix);
    }
    return ds;
}

/* How a render reports its timings: not at all, synchronously (the call waits
 * for the kernels and fills pt_render_stats), or deferred (HIP events and the
 * device counters accumulate in the device state until pt_render_collect, so
 * the render stays asynchronous on the caller's stream: bench.py's reduce
 * follows it without a host round trip). */
enum class Timing
{
    None,
    Sync,
    Deferred
};

/* Reads the recorded launches and the device counters of ds into st (after the
 * last recorded event completes) and forgets them. */
void collect_timings(DeviceState &ds, pt_render_stats *st)
{
    memset(st, 0, sizeof(*st));
    if (ds.pending.empty())
        return;
    /* renders may have been queued on different streams: wait for each one's
     * last event before reading any elapsed time */
    for (auto &pr : ds.pending)
        HIPCHECK(hipEventSynchronize(pr.evs.back()));
    for (auto &pr : ds.pending) {
        for (auto &sp : pr.spans) {
            float ms = 0;
            HIPCHECK(hipEventElapsedTime(&ms, pr.evs[sp.first], pr.evs[sp.second]));
            st->kernel_ms += ms;
            st->launches++;
        }
        for (auto &sp : pr.rspans) {
            float ms = 0;
            HIPCHECK(hipEventElapsedTime(&ms, pr.evs[sp.first], pr.evs[sp.second]));
            st->reduce_ms += ms;
        }
        st->samples += pr.samples;
    }
    uint64_t c[40];
    HIPCHECK(hipMemcpy(c, ds.stats.p, sizeof c, hipMemcpyDeviceToHost));
    st->queries = c[0] + c[1];
    st->leaf_queries = c[1];
    st->attempts = c[2];
    st->rounds = c[3];
    st->slow_queries = c[6];
    st->dark_queries = c[7];
    st->mid_queries = c[24];
    if (c[29])
        st->wave_ms = (double)c[28] * (double)st->launches / (double)c[29] / 1e5; /* 100 MHz clock */
    if (getenv("PT_PHASE_DUMP")) /* profiling builds (PT_PHASE_TIMING): per-phase wave cycles */
    {
        fprintf(stderr, "pt_phases");
        for (int k = 8; k < 15; k++)
            fprintf(stderr, " %llu", (unsigned long long)c[k]);
        for (int k = 16; k < 24; k++)
            fprintf(stderr, " %llu", (unsigned long long)c[k]);
        fprintf(stderr, " %llu", (unsigned long long)c[25]); /* whole chunk loop */
        fprintf(stderr, " %llu %llu", (unsigned long long)c[30], (unsigned long long)c[31]); /* spine queries */
        fprintf(stderr, " %llu %llu", (unsigned long long)c[32], (unsigned long long)c[33]); /* lane front end, writes */
        fprintf(stderr, " %llu", (unsigned long long)c[34]); /* spine queries that ran the lazy merge */
        fprintf(stderr, "\n");
    }
    st->sphere_tests = st->queries * (uint64_t)ds.pending.back().n_spheres;
    st->plane_tests = st->queries * (uint64_t)ds.pending.back().n_planes;
    for (auto &pr : ds.pending)
        for (auto e : pr.evs) (void)hipEventDestroy(e);
    ds.pending.clear();
}

/* compact: with a pixel list, pixel k's result goes to fb[3k..3k+2] (else to
 * its frame position, fb[3 * pixels[k]]) */
constexpr size_t kMaxPending = 1024; /* deferred renders a device keeps before a collect is required */

/* rays (device memory, 7 floats per slot): the ray-list module of
 * pt_trace_rays renders slot k = ray k instead of a camera pixel */
void render_device(SceneImpl &s, const pt_render_params *p, float *fb, hipStream_t stream, pt_render_stats *st,
                   Timing tm, bool compact = false, const float *rays = nullptr, int64_t ray0 = 0)
{
    std::shared_ptr<const Generated> gp;
    DeviceState &ds = prepare(s, p, gp, rays != nullptr);
    const Generated &g = *gp;
    const long long npix = p->pixels ? (long long)p->npixels : (long long)p->width * p->height;
    /* an untimed render queued while timed ones wait for their collect joins
     * them: its launches are timed too, so the counters the collect reads and
     * the kernel times it sums cover the same renders.  The pending cap binds
     * only renders the caller asked to time: a plain render never fails
     * because of another call's uncollected timings */
    const bool joined = tm == Timing::None && !ds.pending.empty();
    if (joined)
        tm = Timing::Deferred;
    if (tm == Timing::Deferred && !joined && ds.pending.size() >= kMaxPending)
        throw Error(PT_ERR_ARG, "too many timed renders pending: call pt_render_collect");
    if (tm == Timing::Sync) {
        memset(st, 0, sizeof(*st));
        for (auto &pr : ds.pending) /* a synchronous render reports itself alone */
            for (auto e : pr.evs) (void)hipEventDestroy(e);
        ds.pending.clear();
    }
    if (npix == 0)
        return;
    const int *dpix = nullptr;
    if (p->pixels) {
        HIPCHECK(hipMemcpyAsync(ds.pixels.p, p->pixels, (size_t)npix * 4, hipMemcpyHostToDevice, stream));
        dpix = ds.pixels.p;
    }
    const long long per_pass = pass_samples(p, npix);
    const bool timed = tm != Timing::None;
    /* the counters restart with the first recorded render */
    if (!timed || ds.pending.empty())
        HIPCHECK(hipMemsetAsync(ds.stats.p, 0, 40 * 8, stream));
    hipFunction_t fn = p->order == PT_ORDER_REFERENCE ? ds.strict : ds.fast;
    PendingRender pr;
    pr.n_spheres = g.n_spheres, pr.n_planes = g.n_planes;
    struct EvGuard /* events of a render that throws before it is recorded */
    {
        PendingRender &pr;
        bool kept = false;
        ~EvGuard()
        {
            if (!kept)
                for (auto e : pr.evs) (void)hipEventDestroy(e);
        }
    } eg{pr};
    auto event = [&]() {
        hipEvent_t e;
        HIPCHECK(hipEventCreate(&e));
        pr.evs.push_back(e);
        HIPCHECK(hipEventRecord(e, stream));
    };
    for (int s0 = 0; s0 < p->spp; s0 += (int)per_pass) {
        int reduce_mode = 0;
        int nsamp = (int)std::min<long long>(per_pass, p->spp - s0);
        long long n_items = npix * nsamp;
        /* 64 items per dequeue: every lane of the chunk's camera phase busy
         * (same-box A/B: C5 2430 -> 4490 Msamples/s, C3 +0.5 %; round 1: C3
         * 16 -> 32 +2.7 %); a launch too small to give every resident wave a
         * few chunks takes fewer, so one wave does not trace many samples of
         * one expensive pixel while others idle */
        const long long waves = (long long)ds.resident_blocks * ds.wpw;
        static const int chunk_max = [] {
            const char *env = getenv("PT_CHUNK_MAX"); /* experiment hook (1..64) */
            if (!env || !*env)
                return 64;
            fprintf(stderr, "pt: experiment hook PT_CHUNK_MAX=%s active\n", env);
            return std::max(1, std::min(64, atoi(env)));
        }();
        int chunk = chunk_max;
        /* slot-major launches of few samples per pixel (a multi-GPU rank's
         * share: C3 at 8 ranks = 128 per pixel) take 32-sample chunks: a
         * chunk is then half as many samples of one expensive pixel, which
         * shortens the launch's tail (same-box A/B at 128 spp: 147.2 -> 153.3
         * Msamples/s; at 256 spp 64 stays ahead, 156.0 vs 153.2) */
        if (nsamp > 64 && nsamp <= 128)
            chunk = std::min(chunk, 32);
        while (chunk > 1 && n_items / chunk < 4 * waves) chunk /= 2;
        long long chunks = (n_items + chunk - 1) / chunk;
        const int wpw = ds.wpw;
        {
            long long blocks = std::min<long long>(ds.resident_blocks, (chunks + wpw - 1) / wpw);
            long long c0 = 0;
            PtLaunchHost lp;
            memset(&lp, 0, sizeof lp);
            lp.seed = p->seed;
            lp.n_items = n_items;
            lp.chunk0 = c0;
            lp.W = p->width, lp.H = p->height;
            lp.sw = p->screen_w, lp.sh = p->screen_h, lp.dist = p->screen_dist;
            lp.depth = p->depth;
            lp.nsamp = nsamp;
            lp.s0 = p->sample_begin + s0;
            lp.gw = p->grid_width > 0 ? p->grid_width : p->width;
            lp.chunk = chunk;
            /* sample-major item order for launches of up to 64 samples per slot
             * (pt_device.h item_slot) */
            lp.sample_major = nsamp <= 64 ? 1 : 0;
            if (lp.sample_major)
                lp.perm = slot_permutation(npix);
            /* one staged partial per 32-sample block when a chunk is a block */
            lp.block_sums =
                (block_staging(p) && !lp.sample_major && (chunk == 32 || chunk == 64) && nsamp % chunk == 0) ? 1 : 0;
            lp.rays = rays;
            lp.ray0 = ray0;
            lp.grab = grab_chunks(s);
            /* split launch (lane-walk modules, fast order): the light kernel
             * over every chunk, then the full kernel over the ones it left */
            const bool split = ds.light && fn == ds.fast && s.split && split_launches() && chunks < (1ll << 32);
            reduce_mode = p->order == PT_ORDER_REFERENCE ? 0 : lp.block_sums ? 2 : 1;
            ds.stage.ensure((size_t)(lp.block_sums ? npix * (nsamp / 32) * 3 : npix * nsamp * 3));
            const float *Pp = ds.P.p;
            const PtImageDev *ip = ds.imgs.p;
            const uint64_t *jp = ds.jump.p;
            float *op = ds.stage.p;
            const int *pp = dpix;
            uint64_t *sp = ds.stats.p; /* counters + the persistent chunk counter (stats[15]) */
            HIPCHECK(hipMemsetAsync(ds.stats.p + 15, 0, 8, stream));
            void *args[] = {&Pp, &ip, &jp, &op, &pp, &sp, &lp};
            int e0 = (int)pr.evs.size();
            if (timed)
                event();
            if (split) {
                ds.bail.ensure((size_t)chunks);
                HIPCHECK(hipMemsetAsync(ds.stats.p + 35, 0, 16, stream)); /* list length, its queue */
                lp.bail = ds.bail.p;
                const long long lblocks = std::min<long long>(ds.light_blocks, (chunks + wpw - 1) / wpw);
                HIPCHECK(hipModuleLaunchKernel(ds.light, (unsigned)lblocks, 1, 1, 64 * wpw, 1, 1, 0, stream, args,
                                               nullptr));
                lp.bail = nullptr;
                lp.list = ds.bail.p;
            }
            HIPCHECK(hipModuleLaunchKernel(fn, (unsigned)blocks, 1, 1, 64 * wpw, 1, 1, 0, stream, args, nullptr));
            if (timed) {
                event();
                pr.spans.push_back({e0, e0 + 1});
            }
        }
        {
            const float *in = ds.stage.p;
            float *acc = ds.accum.p;
            const int *pp = compact ? nullptr : dpix; /* output index: slot (compact) or pixel */
            long long ns = npix;
            int first = s0 == 0, last = s0 + nsamp == p->spp;
            float spp = p->sum_only ? 1.0f : (float)p->spp; /* x / 1 == x: the raw sum */
            void *args[] = {&in, &acc, &fb, &pp, &ns, &nsamp, &first, &last, &spp, &reduce_mode};
            unsigned blocks = (unsigned)((npix + 255) / 256);
            int e0 = (int)pr.evs.size();
            if (timed)
                event();
            HIPCHECK(hipModuleLaunchKernel(ds.reduce, blocks, 1, 1, 256, 1, 1, 0, stream, args, nullptr));
            if (timed) {
                event();
                pr.rspans.push_back({e0, e0 + 1});
            }
        }
        pr.samples += (uint64_t)n_items;
    }
    if (!timed)
        return;
    eg.kept = true;
    ds.pending.push_back(std::move(pr));
    if (tm == Timing::Sync)
        collect_timings(ds, st);
}

/* A query module (generate_query) loaded on one device with its own copy of
 * the parameters and images; everything is released with it.  A scene keeps
 * the modules it has served (SceneImpl::qcache): a scene only grows, so a
 * module whose source key, parameters and image slots match is the same
 * module, and the facade's per-ray / per-point virtuals (SpanIterator::init,
 * Texture::getColor) reuse it instead of loading a code object per call. */
struct QueryModule
{
    int device;
    hipModule_t mod = nullptr;
    std::vector<float> params;
    std::vector<int> image_ids;
    DevBuf<float> P;
    DevBuf<PtImageDev> imgs;
    std::vector<DevBuf<float>> img_data;
    QueryModule(SceneImpl &s, const Generated &g, int dev) : device(dev), params(g.params), image_ids(g.image_ids)
    {
        const std::vector<char> &code = code_object(g);
        HIPCHECK(hipSetDevice(device));
        HIPCHECK(hipModuleLoadData(&mod, code.data()));
        try {
            P.ensure(g.params.size());
            HIPCHECK(hipMemcpy(P.p, g.params.data(), g.params.size() * 4, hipMemcpyHostToDevice));
            img_data.resize(g.image_ids.size());
            std::vector<PtImageDev> desc(g.image_ids.size() + 1);
            for (size_t k = 0; k < g.image_ids.size(); k++) {
                const ImageRec &im = s.images.at(g.image_ids[k]);
                img_data[k].ensure(im.rgba.size());
                HIPCHECK(hipMemcpy(img_data[k].p, im.rgba.data(), im.rgba.size() * 4, hipMemcpyHostToDevice));
                desc[k].data = img_data[k].p;
                desc[k].w = (uint32_t)im.w;
                desc[k].h = (uint32_t)im.h;
            }
            imgs.ensure(desc.size());
            HIPCHECK(hipMemcpy(imgs.p, desc.data(), desc.size() * sizeof(PtImageDev), hipMemcpyHostToDevice));
        } catch (...) { /* the destructor does not run for a half-built object */
            release();
            throw;
        }
    }
    hipFunction_t fn(const char *name)
    {
        hipFunction_t f;
        HIPCHECK(hipModuleGetFunction(&f, mod, name));
        return f;
    }
    void release()
    {
        P.release(), imgs.release();
        for (auto &b : img_data) b.release();
        if (mod)
            (void)hipModuleUnload(mod);
        mod = nullptr;
    }
    ~QueryModule()
    {
        int prev = 0;
        if (hipGetDevice(&prev) == hipSuccess && hipSetDevice(device) == hipSuccess) {
            release();
            (void)hipSetDevice(prev);
        }
    }
};

/* Restores the calling thread's current HIP device on scope exit. */
struct DeviceGuard
{
    int prev = -1;
    DeviceGuard() { (void)hipGetDevice(&prev); }
    ~DeviceGuard()
    {
        if (prev >= 0)
            (void)hipSetDevice(prev);
    }
};

/* scratch device memory of one query call */
struct Scratch
{
    std::vector<void *> v;
    void *alloc(size_t bytes)
    {
        void *q = nullptr;
        HIPCHECK(hipMalloc(&q, bytes ? bytes : 4));
        v.push_back(q);
        return q;
    }
    ~Scratch()
    {
        for (void *q : v) (void)hipFree(q);
    }
};

} // namespace

/* the scene's loaded query modules, by (source key, device) */
struct QueryCache
{
    std::map<std::pair<std::string, int>, std::unique_ptr<QueryModule>> mods;
};

namespace
{
QueryModule &query_module(SceneImpl &s, const Generated &g, int device)
{
    if (!s.qcache)
        s.qcache = std::shared_ptr<QueryCache>(new QueryCache);
    std::unique_ptr<QueryModule> &q = s.qcache->mods[{g.key, device}];
    if (q && (q->params != g.params || q->image_ids != g.image_ids))
        q.reset();
    if (!q)
        q.reset(new QueryModule(s, g, device));
    HIPCHECK(hipSetDevice(device));
    return *q;
}
} // namespace

} // namespace pt

using namespace pt;

extern "C" {

const char *pt_last_error(void) { return g_error.c_str(); }
const char *pt_version(void) { return "pt-mi355x 0.1 (gfx950)"; }

pt_scene *pt_scene_create(void) { return new pt_scene; }
void pt_scene_destroy(pt_scene *s) { delete s; }

pt_id pt_image_load_hdr(pt_scene *s, const char *path)
{
    return guard([&] {
        SceneImpl &sc = S(s);
        sc.images.push_back(read_hdr(path ? path : ""));
        return (int)sc.images.size() - 1;
    });
}

pt_id pt_image_load_png(pt_scene *s, const char *path)
{
    return guard([&] {
        SceneImpl &sc = S(s);
        sc.images.push_back(read_png(path ? path : ""));
        return (int)sc.images.size() - 1;
    });
}

pt_id pt_image_load(pt_scene *s, const char *path)
{
    return guard([&] {
        SceneImpl &sc = S(s);
        sc.images.push_back(read_image(path ? path : ""));
        return (int)sc.images.size() - 1;
    });
}

pt_id pt_image_from_rgba32f(pt_scene *s, const float *rgba, int w, int h)
{
    return guard([&] {
        SceneImpl &sc = S(s);
        if (!rgba || w <= 0 || h <= 0)
            throw Error(PT_ERR_ARG, "bad image");
        ImageRec r;
        r.w = w, r.h = h;
        r.rgba.assign(rgba, rgba + (size_t)4 * w * h);
        sc.images.push_back(std::move(r));
        return (int)sc.images.size() - 1;
    });
}

int pt_png_read(const char *path, float *rgba, int *w, int *h)
{
    return guard([&] {
        ImageRec r = read_png(path ? path : "");
        if (w)
            *w = r.w;
        if (h)
            *h = r.h;
        if (rgba)
            memcpy(rgba, r.rgba.data(), r.rgba.size() * 4);
        return PT_OK;
    });
}

int pt_hdr_read(const char *path, float *rgba, int *w, int *h)
{
    return guard([&] {
        ImageRec r = read_hdr(path ? path : "");
        if (w)
            *w = r.w;
        if (h)
            *h = r.h;
        if (rgba)
            memcpy(rgba, r.rgba.data(), r.rgba.size() * 4);
        return PT_OK;
    });
}

pt_id pt_tex_color(pt_scene *s, float r, float g, float b)
{
    return guard([&] {
        TexRec t;
        t.kind = TexKind::Color;
        t.f[0] = r, t.f[1] = g, t.f[2] = b;
        return add_tex(S(s), t);
    });
}

static pt_id tex_image(pt_scene *s, TexKind k, pt_id image)
{
    return guard([&] {
        SceneImpl &sc = S(s);
        check_img(sc, image);
        TexRec t;
        t.kind = k;
        t.img[0] = image;
        return add_tex(sc, t);
    });
}
pt_id pt_tex_image(pt_scene *s, pt_id image) { return tex_image(s, TexKind::Image, image); }
pt_id pt_tex_image_alpha(pt_scene *s, pt_id image) { return tex_image(s, TexKind::ImageAlpha, image); }

static pt_id tex_skybox(pt_scene *s, TexKind k, const pt_id *f)
{
    return guard([&] {
        SceneImpl &sc = S(s);
        TexRec t;
        t.kind = k;
        for (int j = 0; j < 6; j++) {
            check_img(sc, f[j]);
            t.img[j] = f[j];
        }
        return add_tex(sc, t);
    });
}
pt_id pt_tex_skybox(pt_scene *s, pt_id top, pt_id bottom, pt_id left, pt_id right, pt_id front, pt_id back)
{
    pt_id f[6] = {top, bottom, left, right, front, back};
    return tex_skybox(s, TexKind::Skybox, f);
}
pt_id pt_tex_skybox_alpha(pt_scene *s, pt_id top, pt_id bottom, pt_id left, pt_id right, pt_id front, pt_id back)
{
    pt_id f[6] = {top, bottom, left, right, front, back};
    return tex_skybox(s, TexKind::SkyboxAlpha, f);
}

static pt_id tex_wrap(pt_scene *s, TexKind k, pt_id inner, const float *f, int nf)
{
    return guard([&] {
        SceneImpl &sc = S(s);
        check_tex(sc, inner);
        TexRec t;
        t.kind = k;
        t.child = inner;
        for (int j = 0; j < nf; j++) t.f[j] = f[j];
        return add_tex(sc, t);
    });
}
pt_id pt_tex_multiply(pt_scene *s, float r, float g, float b, pt_id t)
{
    float f[3] = {r, g, b};
    return tex_wrap(s, TexKind::Multiply, t, f, 3);
}
pt_id pt_tex_log(pt_scene *s, pt_id t) { return tex_wrap(s, TexKind::Log, t, nullptr, 0); }
pt_id pt_tex_mirrorball(pt_scene *s, pt_id t) { return tex_wrap(s, TexKind::MirrorBall, t, nullptr, 0); }
pt_id pt_tex_spherical(pt_scene *s, pt_id t) { return tex_wrap(s, TexKind::Spherical, t, nullptr, 0); }
pt_id pt_tex_transformed(pt_scene *s, const float m[12], pt_id t)
{
    if (!m) {
        set_error("null matrix");
        return PT_ERR_ARG;
    }
    return tex_wrap(s, TexKind::Xform, t, m, 12);
}
pt_id pt_tex_coord(pt_scene *s)
{
    return guard([&] {
        TexRec t;
        t.kind = TexKind::Coord;
        return add_tex(S(s), t);
    });
}

/* A user-defined Texture subclass (include/texture.h:10-27: getColor, and
 * getFloat's default unless overridden) as device source, compiled into every
 * module of the scene that reaches it (codegen.cpp UTex_<id>). */
pt_id pt_tex_device(pt_scene *s, const char *color_body, const char *value_body, const float *params, int nparams)
{
    return guard([&] {
        if (!color_body || !*color_body)
            throw Error(PT_ERR_ARG, "pt_tex_device: empty getColor body");
        if (nparams < 0 || nparams > (1 << 16) || (nparams > 0 && !params))
            throw Error(PT_ERR_ARG, "pt_tex_device: bad parameter block");
        TexRec t;
        t.kind = TexKind::User;
        t.color_body = color_body;
        t.value_body = value_body ? value_body : "";
        t.params.assign(params, params + nparams);
        return add_tex(S(s), t);
    });
}

pt_id pt_material(pt_scene *s, pt_id reflect, pt_id scatter, pt_id emissive, pt_id transmit, float ior,
                  pt_id transmit_reflect)
{
    return guard([&] {
        SceneImpl &sc = S(s);
        /* include/material.h:18 defaults: reflect 1, scatter 1, emissive 0, transmit 0, trc 0 */
        if (reflect < 0)
            reflect = default_tex(sc, 1);
        if (scatter < 0)
            scatter = default_tex(sc, 1);
        if (emissive < 0)
            emissive = default_tex(sc, 0);
        if (transmit < 0)
            transmit = default_tex(sc, 0);
        if (transmit_reflect < 0)
            transmit_reflect = default_tex(sc, 0);
        for (int t : {reflect, scatter, emissive, transmit, transmit_reflect}) check_tex(sc, t);
        MatRec m{reflect, scatter, emissive, transmit, transmit_reflect, ior};
        sc.materials.push_back(m);
        return (int)sc.materials.size() - 1;
    });
}

pt_id pt_sphere(pt_scene *s, float cx, float cy, float cz, float r, pt_id mat)
{
    return guard([&] {
        SceneImpl &sc = S(s);
        check_mat(sc, mat);
        ObjRec o;
        o.kind = ObjKind::Sphere;
        o.f[0] = cx, o.f[1] = cy, o.f[2] = cz, o.f[3] = r;
        o.mat = mat;
        sc.objects.push_back(o);
        return (int)sc.objects.size() - 1;
    });
}

pt_id pt_plane(pt_scene *s, float nx, float ny, float nz, float d, pt_id mat)
{
    return guard([&] {
        SceneImpl &sc = S(s);
        check_mat(sc, mat);
        ObjRec o;
        o.kind = ObjKind::Plane;
        o.f[0] = nx, o.f[1] = ny, o.f[2] = nz, o.f[3] = d;
        o.mat = mat;
        sc.objects.push_back(o);
        return (int)sc.objects.size() - 1;
    });
}

pt_id pt_plane_through(pt_scene *s, float nx, float ny, float nz, float px, float py, float pz, pt_id mat)
{
    /* Plane(normal, pos): d = -dot(normal, pos), src/plane.cpp:11-14 */
    float d = -((nx * px + ny * py) + nz * pz);
    return pt_plane(s, nx, ny, nz, d, mat);
}

pt_id pt_csg(pt_scene *s, int op, pt_id a, pt_id b)
{
    return guard([&] {
        SceneImpl &sc = S(s);
        check_obj(sc, a);
        check_obj(sc, b);
        ObjRec o;
        if (op == PT_CSG_UNION)
            o.kind = ObjKind::Union;
        else if (op == PT_CSG_INTERSECTION)
            o.kind = ObjKind::Intersection;
        else if (op == PT_CSG_DIFFERENCE)
            o.kind = ObjKind::Difference;
        else
            throw Error(PT_ERR_ARG, "bad csg op");
        o.a = a, o.b = b;
        sc.objects.push_back(o);
        return (int)sc.objects.size() - 1;
    });
}

pt_id pt_transformed(pt_scene *s, const float m[12], pt_id child)
{
    return guard([&] {
        SceneImpl &sc = S(s);
        if (!m)
            throw Error(PT_ERR_ARG, "null matrix");
        check_obj(sc, child);
        float inv[12];
        mat_inverse(m, inv); /* the reference inverts in the iterator ctor and throws there */
        ObjRec o;
        o.kind = ObjKind::Xform;
        memcpy(o.f, m, 48);
        o.a = child;
        sc.objects.push_back(o);
        return (int)sc.objects.size() - 1;
    });
}

/* A user-defined Object subclass (include/object.h:10-24: the virtual
 * makeSpanIterator) with one span per ray, as device source compiled into the
 * scene's modules (device/pt_user_object.h). */
pt_id pt_object_device(pt_scene *s, const char *span_body, const char *normal_body, const float *params,
                       int nparams, pt_id mat)
{
    return guard([&] {
        SceneImpl &sc = S(s);
        if (!span_body || !*span_body || !normal_body || !*normal_body)
            throw Error(PT_ERR_ARG, "pt_object_device: empty span or normal body");
        if (nparams < 0 || nparams > (1 << 16) || (nparams > 0 && !params))
            throw Error(PT_ERR_ARG, "pt_object_device: bad parameter block");
        check_mat(sc, mat);
        ObjRec o;
        o.kind = ObjKind::User;
        o.mat = mat;
        o.span_body = span_body;
        o.normal_body = normal_body;
        o.params.assign(params, params + nparams);
        sc.objects.push_back(o);
        return (int)sc.objects.size() - 1;
    });
}

int pt_set_root(pt_scene *s, pt_id obj)
{
    return guard([&] {
        SceneImpl &sc = S(s);
        check_obj(sc, obj);
        sc.root = obj;
        return PT_OK;
    });
}

int pt_scene_from_text(pt_scene *s, const char *text)
{
    return guard([&] {
        load_text(S(s), text ? text : "");
        return PT_OK;
    });
}

void pt_matrix_rotate(const float axis[3], double angle, float out[12]) { mat_rotate(axis, angle, out); }
int pt_matrix_inverse(const float m[12], float out[12])
{
    return guard([&] {
        mat_inverse(m, out);
        return PT_OK;
    });
}
void pt_matrix_concat(const float a[12], const float b[12], float out[12]) { mat_concat(a, b, out); }

int pt_scene_compile(pt_scene *s, int depth)
{
    return guard([&] {
        Generated g = generate(S(s), depth);
        code_object(g);
        S(s).last_key = g.key;
        return PT_OK;
    });
}

int pt_scene_set_occupancy(pt_scene *s, int workgroups_per_cu)
{
    return guard([&] {
        if (workgroups_per_cu < 0 || workgroups_per_cu > 5)
            throw Error(PT_ERR_ARG, "workgroups_per_cu must be 0 (auto) or 1..5");
        S(s).wg_per_cu = workgroups_per_cu;
        return PT_OK;
    });
}

int pt_scene_set_fast_spine(pt_scene *s, int on)
{
    return guard([&] {
        S(s).fast_spine = on ? 1 : 0;
        return PT_OK;
    });
}

int pt_scene_set_lane_walk(pt_scene *s, int frames)
{
    return guard([&] {
        if (frames < 0 || frames > 8)
            throw Error(PT_ERR_ARG, "lane walk frames must be in [0, 8]");
        S(s).lane_walk = frames;
        return PT_OK;
    });
}

int pt_scene_set_split(pt_scene *s, int on)
{
    return guard([&] {
        S(s).split = on ? 1 : 0;
        return PT_OK;
    });
}

int pt_scene_set_lane_scatter(pt_scene *s, int on)
{
    return guard([&] {
        S(s).lane_scatter = on ? 1 : 0;
        return PT_OK;
    });
}

const char *pt_scene_kernel_key(pt_scene *s, int depth)
{
    thread_local std::string k;
    try {
        k = code_object_key(generate(S(s), depth));
    } catch (std::exception &e) {
        set_error(e.what());
        k.clear();
    }
    return k.c_str();
}

int pt_prepare(pt_scene *s, const pt_render_params *p)
{
    return guard([&] {
        std::shared_ptr<const Generated> g;
        prepare(S(s), p, g);
        return PT_OK;
    });
}

int pt_render_device(pt_scene *s, const pt_render_params *p, float *fb, void *stream, pt_render_stats *stats)
{
    return guard([&] {
        if (!fb)
            throw Error(PT_ERR_ARG, "null frame buffer");
        render_device(S(s), p, fb, (hipStream_t)stream, stats, stats ? Timing::Sync : Timing::None);
        return PT_OK;
    });
}

int pt_render_device_timed(pt_scene *s, const pt_render_params *p, float *fb, void *stream)
{
    return guard([&] {
        if (!fb)
            throw Error(PT_ERR_ARG, "null frame buffer");
        render_device(S(s), p, fb, (hipStream_t)stream, nullptr, Timing::Deferred);
        return PT_OK;
    });
}

int pt_render_collect(pt_scene *s, int device, pt_render_stats *stats)
{
    return guard([&] {
        if (!stats)
            throw Error(PT_ERR_ARG, "null stats");
        SceneImpl &sc = S(s);
        auto it = sc.devices.find(device);
        if (it == sc.devices.end() || !it->second) {
            memset(stats, 0, sizeof(*stats));
            return PT_OK;
        }
        HIPCHECK(hipSetDevice(device));
        collect_timings(*it->second, stats);
        return PT_OK;
    });
}

constexpr size_t kPinFloats = (size_t)1 << 20; /* results up to 4 MB go through pinned staging */

int pt_render(pt_scene *s, const pt_render_params *p, float *rgb_out, pt_render_stats *stats)
{
    const double t0 = now_us();
    for (double &v : g_prof) v = 0.0;
    return guard([&] {
        if (!rgb_out)
            throw Error(PT_ERR_ARG, "null output");
        validate(p);
        SceneImpl &sc = S(s);
        HIPCHECK(hipSetDevice(p->device));
        /* a pixel list renders into a compact buffer, pixel k at 3k; pt_reduce
         * writes every slot of it, so the buffer needs no clearing */
        const size_t n = p->pixels ? (size_t)std::max<int64_t>(1, p->npixels) * 3 : frame_floats(p);
        std::shared_ptr<const Generated> gp;
        DeviceState &ds = prepare(sc, p, gp, false);
        ds.out.ensure(n);
        const size_t nout = p->pixels ? (size_t)p->npixels * 3 : n;
        /* small calls (a pixel, a block) stage the pixel list and the result in
         * pinned memory: asynchronous DMA both ways and one synchronisation */
        const bool pin = nout <= kPinFloats;
        pt_render_params q = *p;
        if (pin && p->pixels && p->npixels > 0) {
            ds.hpix.ensure((size_t)p->npixels);
            memcpy(ds.hpix.p, p->pixels, (size_t)p->npixels * 4);
            q.pixels = ds.hpix.p;
        }
        if (pin)
            ds.hout.ensure(std::max<size_t>(nout, 1));
        const double t1 = now_us();
        /* without stats the launches carry no events and no counter read-back */
        pt_render_stats local;
        const bool want = stats != nullptr || getenv("PT_CALL_KERNEL_TIME");
        render_device(sc, &q, ds.out.p, nullptr, stats ? stats : &local, want ? Timing::Sync : Timing::None, true);
        if (pin && nout)
            HIPCHECK(hipMemcpyAsync(ds.hout.p, ds.out.p, nout * 4, hipMemcpyDeviceToHost, nullptr));
        const double t2 = now_us();
        HIPCHECK(hipStreamSynchronize(nullptr));
        const double t3 = now_us();
        if (nout) {
            if (pin)
                memcpy(rgb_out, ds.hout.p, nout * 4);
            else
                HIPCHECK(hipMemcpy(rgb_out, ds.out.p, nout * 4, hipMemcpyDeviceToHost));
        }
        const double t4 = now_us();
        g_prof[PT_PROF_SETUP] = t1 - t0;
        g_prof[PT_PROF_ENQUEUE] = t2 - t1;
        g_prof[PT_PROF_WAIT] = t3 - t2;
        g_prof[PT_PROF_D2H] = t4 - t3;
        g_prof[PT_PROF_TOTAL] = t4 - t0;
        if (want) {
            const pt_render_stats &st = stats ? *stats : local;
            g_prof[PT_PROF_KERNEL] = st.kernel_ms * 1e3;
            g_prof[PT_PROF_REDUCE] = st.reduce_ms * 1e3;
        }
        return PT_OK;
    });
}

int pt_rank_pixels(int width, int height, int rank, int world, int tile, int32_t *pixels, int64_t capacity,
                   int64_t *count)
{
    return guard([&] {
        if (width <= 0 || height <= 0 || (int64_t)width * height >= (1ll << 31))
            throw Error(PT_ERR_ARG, "bad frame size");
        if (world < 1 || rank < 0 || rank >= world || tile < 1)
            throw Error(PT_ERR_ARG, "need 0 <= rank < world and tile >= 1");
        if (!count || (pixels && capacity < 0))
            throw Error(PT_ERR_ARG, "null count or negative capacity");
        int64_t n = 0;
        for (int y = 0; y < height; y++)
            for (int x = 0; x < width; x++) {
                const int64_t owner = world == 1 ? 0 : ((int64_t)(x / tile) + 3ll * (y / tile)) % world;
                if (owner != rank)
                    continue;
                if (pixels && n < capacity)
                    pixels[n] = y * width + x;
                n++;
            }
        *count = n;
        if (pixels && n > capacity)
            throw Error(PT_ERR_ARG, "capacity below the rank's pixel count");
        return PT_OK;
    });
}

int pt_call_profile(double *out, int n)
{
    if (!out || n < 0)
        return PT_ERR_ARG;
    for (int k = 0; k < n && k < PT_PROF_N; k++) out[k] = g_prof[k];
    return PT_OK;
}

/* traceRay<T>(ray, spanIterator, depth, engine, strength), include/path-trace.h:
 * 58-165, for n caller rays in one launch of the ray-list module: the render
 * kernel with slot k = ray k (origin, direction, strength) instead of a camera
 * ray, spp samples per ray keyed (seed, k, sample), summed in the call's order
 * and divided by spp -- tracePixel's float-coordinate overload (:172-185) when
 * every sample traces the same ray. */
static pt_render_params trace_params(const pt_trace_params *tp, int64_t n)
{
    if (!tp)
        throw Error(PT_ERR_ARG, "null params");
    if (n < 0 || n >= (1ll << 31))
        throw Error(PT_ERR_ARG, "ray count must be in [0, 2^31)");
    if (tp->ray_begin < 0 || tp->ray_begin + n > (1ll << 43))
        throw Error(PT_ERR_ARG, "ray keys must lie in [0, 2^43) (engine key layout)");
    pt_render_params p;
    memset(&p, 0, sizeof p);
    p.width = (int)std::max<int64_t>(1, n), p.height = 1;
    p.spp = tp->spp, p.depth = tp->depth;
    p.screen_w = p.screen_h = p.screen_dist = 1.0f; /* unused: no camera */
    p.seed = tp->seed, p.order = tp->order, p.device = tp->device;
    p.max_buffer_bytes = tp->max_buffer_bytes;
    p.sample_begin = tp->sample_begin;
    return p;
}

int pt_trace_rays(pt_scene *s, const pt_trace_params *tp, const float *rays, int64_t n, float *rgb_out,
                  pt_render_stats *stats)
{
    return guard([&] {
        pt_render_params p = trace_params(tp, n);
        validate(&p);
        if (n == 0) {
            if (stats)
                memset(stats, 0, sizeof(*stats));
            return PT_OK;
        }
        if (!rays || !rgb_out)
            throw Error(PT_ERR_ARG, "null rays or output");
        for (int64_t k = 0; k < n; k++) {
            /* Ray(o, d) asserts d != 0 (include/ray.h:17) */
            if (rays[7 * k + 3] == 0.0f && rays[7 * k + 4] == 0.0f && rays[7 * k + 5] == 0.0f)
                throw Error(PT_ERR_ARG, "ray " + std::to_string(k) + " has a zero direction");
            /* The kernel's axis-aligned plane forms take d.n as the one product
             * that survives for finite operands (the other terms are +-0); an
             * infinite or NaN component would make the reference's full dot
             * product NaN where the device has a number, so such rays are
             * refused rather than traced differently. */
            for (int c = 0; c < 6; c++)
                if (!std::isfinite(rays[7 * k + c]))
                    throw Error(PT_ERR_ARG, "ray " + std::to_string(k) + " has a non-finite origin or direction");
        }
        SceneImpl &sc = S(s);
        HIPCHECK(hipSetDevice(p.device));
        DevBuf<float> fb, rb;
        struct Free
        {
            DevBuf<float> &a, &b;
            ~Free() { a.release(), b.release(); }
        } fr{fb, rb};
        fb.ensure((size_t)n * 3);
        rb.ensure((size_t)n * 7);
        HIPCHECK(hipMemcpy(rb.p, rays, (size_t)n * 7 * 4, hipMemcpyHostToDevice));
        pt_render_stats local;
        render_device(sc, &p, fb.p, nullptr, stats ? stats : &local, Timing::Sync, true, rb.p, tp->ray_begin);
        HIPCHECK(hipDeviceSynchronize());
        HIPCHECK(hipMemcpy(rgb_out, fb.p, (size_t)n * 3 * 4, hipMemcpyDeviceToHost));
        return PT_OK;
    });
}

int pt_trace_compile(pt_scene *s, int depth)
{
    return guard([&] {
        Generated g = generate(S(s), depth, true);
        code_object(g);
        return PT_OK;
    });
}

namespace
{
/* ---- adaptive caller (reference src/test.cpp:40-50, :324-507) ------------ */
struct AV /* Color arithmetic of include/vector3d.h, float, no contraction */
{
    float x, y, z;
};
AV av_add(AV a, AV b) { return {a.x + b.x, a.y + b.y, a.z + b.z}; }
AV av_sub(AV a, AV b) { return {a.x - b.x, a.y - b.y, a.z - b.z}; }
AV av_scale(float s, AV a) { return {a.x * s, a.y * s, a.z * s}; } /* operator*(float, V) = V * s */
float av_abs2(AV a) { return (a.x * a.x + a.y * a.y) + a.z * a.z; }

int demo_block_size(int count) /* getBlockSize, src/test.cpp:40-48 */
{
    int r = 1024;
    while (r > count && r > 4) r /= 2;
    return r / 4;
}

/* RenderBlock's (size+1)^2 pixel cache (src/test.cpp:396-422), with the
 * traced and interpolated pixels kept apart (state 1 / 2): depth-first, a
 * square left of / above an interpolated neighbour reads that neighbour's
 * left / top edge before the interpolation overwrites it, so calc must see
 * the traced value while the image keeps the interpolated one. */
struct ABlock
{
    int x0, y0, S;
    std::vector<AV> buf;
    std::vector<char> st; /* 0 unset, 1 traced, 2 interpolated */
    bool in(int x, int y) const { return x >= x0 && x - x0 <= S && y >= y0 && y - y0 <= S; }
    size_t at(int x, int y) const { return (size_t)(x - x0) + (size_t)(y - y0) * (S + 1); }
    bool traced(int x, int y) const { return in(x, y) && st[at(x, y)] == 1; }
    void set_traced(int x, int y, AV c)
    {
        if (in(x, y) && st[at(x, y)] != 2)
            buf[at(x, y)] = c, st[at(x, y)] = 1;
    }
    void set_interp(int x, int y, AV c)
    {
        if (in(x, y))
            buf[at(x, y)] = c, st[at(x, y)] = 2;
    }
};

struct ASquare
{
    int b, x, y, size;
    AV tl, tr, bl, br;
};
} // namespace

/* One level-synchronous evaluation of renderSquare over every block: the
 * squares of a level are decided, the points they need are traced in one GPU
 * batch, then their quadrants form the next level.  With traced and
 * interpolated pixels kept apart (ABlock), every calcPixelColor sees what it
 * sees depth-first -- the traced value -- and every interpolation overwrites
 * as it does depth-first, so the image equals the recursion's (checked
 * against the oracle's depth-first restatement, tests/test_adaptive.py). */
int pt_render_adaptive(pt_scene *s, const pt_render_params *p, pt_adaptive_params *ap, float *rgb_out,
                       pt_render_stats *stats)
{
    return guard([&] {
        if (!rgb_out || !ap)
            throw Error(PT_ERR_ARG, "null output or adaptive params");
        if (p->pixels)
            throw Error(PT_ERR_ARG, "adaptive render takes no pixel list");
        if (p->sum_only)
            throw Error(PT_ERR_ARG, "adaptive render interpolates means: sum_only is not supported");
        validate(p);
        (void)S(s);
        const int W = p->width, H = p->height;
        const int S = ap->block_size > 0 ? ap->block_size : demo_block_size(W / 8);
        /* blocks reach x = ceil(W / S) * S: the engine grid is that wide + 1 */
        const int gw = (W + S - 1) / S * S + 1;
        const int maxS = ap->max_interp > 0 ? ap->max_interp : H / (480 / 4);
        const float mcd = ap->min_delta > 0 ? ap->min_delta : 0.003f;
        if (S <= 0)
            throw Error(PT_ERR_ARG, "block size must be positive");
        std::vector<ABlock> blocks;
        for (int y0 = 0; y0 < H; y0 += S) /* makeBlockRenderer order, src/test.cpp:940-956 */
            for (int x0 = 0; x0 < W; x0 += S) {
                ABlock b{x0, y0, S, std::vector<AV>((size_t)(S + 1) * (S + 1)),
                         std::vector<char>((size_t)(S + 1) * (S + 1), 0)};
                blocks.push_back(std::move(b));
            }
        struct TP
        {
            AV c;
            bool used;
        };
        std::map<int64_t, TP> traced;
        std::vector<int32_t> need;
        /* Lookahead: a batch that runs anyway also traces the next level's
         * possible points (the five midpoints of every square the next level
         * could split), so the level after it usually needs no batch of its
         * own -- half the launches, each of which waits on its slowest sample.
         * A point's colour depends only on its (x, y) and the sample indices,
         * never on the batch, so the image is the same bits either way. */
        static const int lookahead_levels = [] {
            const char *env = getenv("PT_ADAPTIVE_LOOKAHEAD"); /* experiment hook: levels traced ahead */
            if (!env || !*env)
                return 2; /* C3 16 spp: 1 -> 3 batches 483 ms, 2 -> 2 batches 436 ms, 3 -> 2 batches 466 ms */
            fprintf(stderr, "pt: experiment hook PT_ADAPTIVE_LOOKAHEAD=%s active\n", env);
            return std::max(1, std::min(4, atoi(env)));
        }();
        const int LA = ap->exact_batches == 0 ? lookahead_levels : 0;
        pt_render_stats acc;
        memset(&acc, 0, sizeof acc);
        ap->traced_pixels = 0;
        ap->lookahead_pixels = 0;
        ap->levels = 0;
        auto want = [&](int x, int y) {
            const int64_t k = (int64_t)y * gw + x;
            if (k < 0 || k > INT32_MAX)
                throw Error(PT_ERR_ARG, "adaptive block reaches past the index range");
            if (traced.emplace(k, TP{AV{0, 0, 0}, false}).second)
                need.push_back((int32_t)k);
        };
        auto flush = [&]() {
            if (need.empty())
                return;
            pt_render_params q = *p;
            q.pixels = need.data();
            q.npixels = (int64_t)need.size();
            q.grid_width = gw;
            std::vector<float> out(need.size() * 3);
            pt_render_stats st;
            int rc = pt_render(s, &q, out.data(), &st);
            if (rc != PT_OK)
                throw Error(rc, pt_last_error());
            for (size_t k = 0; k < need.size(); k++)
                traced[need[k]].c = AV{out[3 * k], out[3 * k + 1], out[3 * k + 2]};
            acc.kernel_ms += st.kernel_ms, acc.reduce_ms += st.reduce_ms, acc.launches += st.launches;
            acc.samples += st.samples, acc.queries += st.queries, acc.leaf_queries += st.leaf_queries;
            acc.attempts += st.attempts, acc.rounds += st.rounds, acc.slow_queries += st.slow_queries;
            acc.dark_queries += st.dark_queries, acc.mid_queries += st.mid_queries;
            acc.wave_ms += st.wave_ms; /* summed over the batches, like kernel_ms */
            ap->levels++;
            need.clear();
        };
        /* calcPixelColor (src/test.cpp:441-465): the block's cached pixel, else the trace */
        auto calc = [&](ABlock &b, int x, int y) {
            if (b.traced(x, y))
                return b.buf[b.at(x, y)];
            TP &t = traced.at((int64_t)y * gw + x);
            t.used = true;
            b.set_traced(x, y, t.c);
            return t.c;
        };
        /* the five points a square's split traces (renderSquare, :478-491) */
        auto mids = [&](int x, int y, int size, const ABlock &b) {
            const int h = size / 2, cx = x + h, cy = y + h;
            const int pts[5][2] = {{cx, y}, {x, cy}, {cx, cy}, {x + size, cy}, {cx, y + size}};
            for (const auto &pt : pts)
                if (!b.traced(pt[0], pt[1]))
                    want(pt[0], pt[1]);
        };
        /* the next levels' possible points: the midpoints of every square of
         * size `size` at (x, y) that a level could split, `levels` deep */
        std::function<void(int, int, int, const ABlock &, int)> ahead = [&](int x, int y, int size,
                                                                           const ABlock &b, int levels) {
            if (levels <= 0 || size <= 1 || x > W || y > H)
                return;
            mids(x, y, size, b);
            const int h = size / 2;
            ahead(x, y, h, b, levels - 1), ahead(x + h, y, h, b, levels - 1), ahead(x, y + h, h, b, levels - 1),
                ahead(x + h, y + h, h, b, levels - 1);
        };
        for (ABlock &b : blocks) {
            want(b.x0, b.y0), want(b.x0 + S, b.y0), want(b.x0, b.y0 + S), want(b.x0 + S, b.y0 + S);
        }
        for (ABlock &b : blocks)
            ahead(b.x0, b.y0, S, b, LA);
        flush();
        std::vector<ASquare> cur;
        for (size_t i = 0; i < blocks.size(); i++) { /* RenderBlock::run, :501-507 */
            ABlock &b = blocks[i];
            AV tl = calc(b, b.x0, b.y0), tr = calc(b, b.x0 + S, b.y0), bl = calc(b, b.x0, b.y0 + S),
               br = calc(b, b.x0 + S, b.y0 + S);
            cur.push_back({(int)i, b.x0, b.y0, S, tl, tr, bl, br});
        }
        const float mcd2 = mcd * mcd;
        auto close = [&](AV a, AV c) { return av_abs2(av_sub(a, c)) <= mcd2 * av_abs2(a); };
        while (!cur.empty()) { /* renderSquare, :466-499 */
            std::vector<ASquare> split;
            for (const ASquare &q : cur) {
                ABlock &b = blocks[q.b];
                if (q.x > W || q.y > H)
                    continue;
                if (q.size <= 1) {
                    b.set_traced(q.x, q.y, q.tl);
                    continue;
                }
                if (close(q.tl, q.tr) && close(q.tl, q.bl) && close(q.tl, q.br) && close(q.tr, q.bl) &&
                    close(q.tr, q.br) && close(q.bl, q.br) && q.size <= maxS) {
                    for (int yy = 0; yy < q.size; yy++) { /* interpolateSquare, :423-436 */
                        const float fy = (float)yy / q.size;
                        const AV l = av_add(q.tl, av_scale(fy, av_sub(q.bl, q.tl)));
                        const AV r = av_add(q.tr, av_scale(fy, av_sub(q.br, q.tr)));
                        for (int xx = 0; xx < q.size; xx++) {
                            const float fx = (float)xx / q.size;
                            b.set_interp(xx + q.x, yy + q.y, av_add(l, av_scale(fx, av_sub(r, l))));
                        }
                    }
                    continue;
                }
                mids(q.x, q.y, q.size, b);
                split.push_back(q);
            }
            /* a batch runs for this level: add the next level's possible points */
            if (!need.empty())
                for (const ASquare &q : split) {
                    const int h = q.size / 2, cx = q.x + h, cy = q.y + h;
                    const ABlock &b = blocks[q.b];
                    ahead(q.x, q.y, h, b, LA), ahead(cx, q.y, h, b, LA), ahead(q.x, cy, h, b, LA),
                        ahead(cx, cy, h, b, LA);
                }
            flush();
            std::vector<ASquare> next;
            for (const ASquare &q : split) {
                ABlock &b = blocks[q.b];
                const int h = q.size / 2, cx = q.x + h, cy = q.y + h;
                const AV tc = calc(b, cx, q.y), cl = calc(b, q.x, cy), cc = calc(b, cx, cy),
                         cr = calc(b, q.x + q.size, cy), bc = calc(b, cx, q.y + q.size);
                next.push_back({q.b, q.x, q.y, h, q.tl, tc, cl, cc});
                next.push_back({q.b, cx, q.y, h, tc, q.tr, cc, cr});
                next.push_back({q.b, q.x, cy, h, cl, cc, q.bl, bc});
                next.push_back({q.b, cx, cy, h, cc, cr, bc, q.br});
            }
            cur.swap(next);
        }
        for (const auto &kv : traced)
            (kv.second.used ? ap->traced_pixels : ap->lookahead_pixels)++;
        /* copyToBuffer, :362-374: each block's interior, valid pixels only */
        std::fill(rgb_out, rgb_out + (size_t)W * H * 3, 0.0f);
        for (const ABlock &b : blocks)
            for (int y = b.y0; y < b.y0 + S && y < H; y++)
                for (int x = b.x0; x < b.x0 + S && x < W; x++)
                    if (b.st[b.at(x, y)]) {
                        const AV c = b.buf[b.at(x, y)];
                        float *o = rgb_out + 3 * ((size_t)y * W + x);
                        o[0] = c.x, o[1] = c.y, o[2] = c.z;
                    }
        if (stats)
            *stats = acc;
        return PT_OK;
    });
}

int pt_query_spans(pt_scene *s, pt_id obj, const float *rays, int64_t n, int max_spans, pt_span *out,
                   int32_t *counts, int device)
{
    return guard([&] {
        SceneImpl &sc = S(s);
        if (obj < 0)
            obj = sc.root;
        check_obj(sc, obj);
        if (n < 0 || max_spans < 0 || (n > 0 && (!rays || !counts || (max_spans > 0 && !out))))
            throw Error(PT_ERR_ARG, "bad query arguments");
        if (n == 0)
            return PT_OK;
        static_assert(sizeof(pt_span) == 40, "pt_span is ten 4-byte words");
        Generated g = generate_query(sc, obj, -1);
        DeviceGuard dg;
        QueryModule &q = query_module(sc, g, device);
        Scratch sm;
        float *dr = (float *)sm.alloc((size_t)n * 24);
        float *dout = (float *)sm.alloc((size_t)n * std::max(1, max_spans) * 40);
        int *dc = (int *)sm.alloc((size_t)n * 4);
        HIPCHECK(hipMemcpy(dr, rays, (size_t)n * 24, hipMemcpyHostToDevice));
        const float *Pp = q.P.p;
        const PtImageDev *ip = q.imgs.p;
        long long nn = n;
        int ms = max_spans;
        void *args[] = {&Pp, &ip, &dr, &nn, &ms, &dout, &dc};
        HIPCHECK(hipModuleLaunchKernel(q.fn("pt_query_spans"), (unsigned)((n + 255) / 256), 1, 1, 256, 1, 1, 0,
                                       nullptr, args, nullptr));
        HIPCHECK(hipDeviceSynchronize());
        HIPCHECK(hipMemcpy(counts, dc, (size_t)n * 4, hipMemcpyDeviceToHost));
        if (max_spans > 0) {
            HIPCHECK(hipMemcpy(out, dout, (size_t)n * max_spans * 40, hipMemcpyDeviceToHost));
            /* compact material indices -> the scene's material ids */
            for (int64_t i = 0; i < n; i++)
                for (int c = 0; c < std::min<int>(counts[i], max_spans); c++) {
                    pt_span &sp = out[i * max_spans + c];
                    sp.mat_start = g.mat_ids.at((size_t)sp.mat_start);
                    sp.mat_end = g.mat_ids.at((size_t)sp.mat_end);
                }
        }
        return PT_OK;
    });
}

int pt_tex_eval(pt_scene *s, pt_id tex, const float *points, int64_t n, float *rgb, float *value, int device)
{
    return guard([&] {
        SceneImpl &sc = S(s);
        check_tex(sc, tex);
        if (n < 0 || (n > 0 && (!points || !rgb || !value)))
            throw Error(PT_ERR_ARG, "bad texture query arguments");
        if (n == 0)
            return PT_OK;
        Generated g = generate_query(sc, -1, tex);
        DeviceGuard dg;
        QueryModule &q = query_module(sc, g, device);
        Scratch sm;
        float *dp = (float *)sm.alloc((size_t)n * 12), *dc = (float *)sm.alloc((size_t)n * 12);
        float *dv = (float *)sm.alloc((size_t)n * 4);
        HIPCHECK(hipMemcpy(dp, points, (size_t)n * 12, hipMemcpyHostToDevice));
        const float *Pp = q.P.p;
        const PtImageDev *ip = q.imgs.p;
        long long nn = n;
        void *args[] = {&Pp, &ip, &dp, &nn, &dc, &dv};
        HIPCHECK(hipModuleLaunchKernel(q.fn("pt_tex_eval"), (unsigned)((n + 255) / 256), 1, 1, 256, 1, 1, 0, nullptr,
                                       args, nullptr));
        HIPCHECK(hipDeviceSynchronize());
        HIPCHECK(hipMemcpy(rgb, dc, (size_t)n * 12, hipMemcpyDeviceToHost));
        HIPCHECK(hipMemcpy(value, dv, (size_t)n * 4, hipMemcpyDeviceToHost));
        return PT_OK;
    });
}

/* Compile (or fetch from the cache) the query module of pt_query_spans /
 * pt_tex_eval without a device. */
int pt_query_compile(pt_scene *s, pt_id obj, pt_id tex)
{
    return guard([&] {
        SceneImpl &sc = S(s);
        if (obj >= 0)
            check_obj(sc, obj);
        if (tex >= 0)
            check_tex(sc, tex);
        /* obj -1: the root (unless only a texture is asked for); obj -2: no object */
        if (obj == -1 && tex < 0)
            obj = sc.root, check_obj(sc, obj);
        (void)code_object(generate_query(sc, obj < 0 ? -1 : obj, tex));
        return PT_OK;
    });
}

/* Runs the device self-test of the exact sqrt/div fast paths on n inputs;
 * mismatches[0..2] = sqrt, div, normalize mismatch counts (all 0 expected). */
int pt_selftest_math(int device, uint64_t n, uint64_t seed, uint64_t *mismatches)
{
    return guard([&] {
        if (!mismatches)
            throw Error(PT_ERR_ARG, "null mismatches");
        Generated g;
        g.source = "#define PT_SELFTEST 1\n" + device_library_source();
        g.key = "selftest";
        const std::vector<char> &code = code_object(g);
        HIPCHECK(hipSetDevice(device));
        hipModule_t mod;
        HIPCHECK(hipModuleLoadData(&mod, code.data()));
        hipFunction_t fn;
        HIPCHECK(hipModuleGetFunction(&fn, mod, "pt_selftest_math"));
        uint64_t *bad = nullptr;
        HIPCHECK(hipMalloc((void **)&bad, 32));
        HIPCHECK(hipMemset(bad, 0, 32));
        void *args[] = {&n, &seed, &bad};
        HIPCHECK(hipModuleLaunchKernel(fn, 4096, 1, 1, 256, 1, 1, 0, nullptr, args, nullptr));
        HIPCHECK(hipDeviceSynchronize());
        HIPCHECK(hipMemcpy(mismatches, bad, 24, hipMemcpyDeviceToHost));
        (void)hipFree(bad);
        (void)hipModuleUnload(mod);
        return PT_OK;
    });
}

/* The device's restated glibc float libm on n operand pairs (pt_device.h
 * pt_selftest_libm): out = n x (atan2f(y, x), asinf(y), logf(x)). */
int pt_selftest_libm(int device, const float *ops, int64_t n, float *out)
{
    return guard([&] {
        if (!ops || !out || n < 0)
            throw Error(PT_ERR_ARG, "bad arguments");
        Generated g;
        g.source = "#define PT_SELFTEST 1\n" + device_library_source();
        g.key = "selftest";
        const std::vector<char> &code = code_object(g);
        HIPCHECK(hipSetDevice(device));
        hipModule_t mod;
        HIPCHECK(hipModuleLoadData(&mod, code.data()));
        struct Unload
        {
            hipModule_t m;
            ~Unload() { (void)hipModuleUnload(m); }
        } ul{mod};
        hipFunction_t fn;
        HIPCHECK(hipModuleGetFunction(&fn, mod, "pt_selftest_libm"));
        DevBuf<float> d_ops, d_out;
        struct Free
        {
            DevBuf<float> &a, &b;
            ~Free() { a.release(), b.release(); }
        } fr{d_ops, d_out};
        d_ops.ensure((size_t)std::max<int64_t>(1, 2 * n));
        d_out.ensure((size_t)std::max<int64_t>(1, 3 * n));
        if (n) {
            HIPCHECK(hipMemcpy(d_ops.p, ops, (size_t)n * 8, hipMemcpyHostToDevice));
            uint64_t nn = (uint64_t)n;
            void *args[] = {&d_ops.p, &nn, &d_out.p};
            HIPCHECK(hipModuleLaunchKernel(fn, 1024, 1, 1, 256, 1, 1, 0, nullptr, args, nullptr));
            HIPCHECK(hipDeviceSynchronize());
            HIPCHECK(hipMemcpy(out, d_out.p, (size_t)n * 12, hipMemcpyDeviceToHost));
        }
        return PT_OK;
    });
}

int pt_write_hdr(const char *path, const float *rgb, int w, int h)
{
    return guard([&] {
        if (!path || !rgb || w <= 0 || h <= 0)
            throw Error(PT_ERR_ARG, "bad arguments");
        write_hdr(path, rgb, w, h);
        return PT_OK;
    });
}

int pt_write_bmp(const char *path, const float *rgb, int w, int h, int count)
{
    return guard([&] {
        if (!path || !rgb || w <= 0 || h <= 0 || count <= 0)
            throw Error(PT_ERR_ARG, "bad arguments");
        write_bmp(path, rgb, w, h, count);
        return PT_OK;
    });
}

} // extern "C"
