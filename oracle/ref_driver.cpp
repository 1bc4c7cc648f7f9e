/*
 * ref_driver.cpp -- TEST INFRASTRUCTURE ONLY.  A driver that is compiled
 * against the UNMODIFIED reference sources where they lie
 * (/root/reference/src/*.cpp + /root/reference/include, see oracle/Makefile)
 * and runs the reference's own hot path so that its outputs can be frozen
 * into tests/golden/ and timed as the CPU baseline ("kind": "reference").
 *
 * It contains no reference code: it builds scenes through the reference's
 * public constructors (Sphere, Plane, Union, Intersection, Difference,
 * TransformedObject, Material, *Texture), then calls
 *   PathTrace::tracePixel<PtSampleEngine>(SpanIterator&, int px, int py, int W, int H,
 *                                         1, depth, sw, sh, dist, engine)
 * (reference include/path-trace.h:187-201) once per (pixel, sample) with the
 * per-sample engine of include/pt/pt_engine.h, summing samples in order and
 * dividing by spp -- the same arithmetic as tracePixel's own spp loop.
 * Threads mirror the reference's block farm (src/test.cpp:147-308, :501-507):
 * every worker owns one SpanIterator from world->makeSpanIterator().
 *
 * Modes (argv[1]):
 *   render  scene.txt W H spp depth sw sh dist seed pixels.bin|all threads per_sample out.bin
 *   spans   scene.txt rays.bin out.bin       full span list of root for each ray
 *   rays    scene.txt rays.bin spp depth seed threads out.bin
 *           traceRay<PtSampleEngine>(ray, it, depth, engine, strength) (path-trace.h:58-165)
 *           per (ray, sample) of rays.bin (n * 7 floats: origin, dir, strength),
 *           Color(0,0,0) + traceRay, summed in sample order, / spp
 *   tex     scene.txt points.bin out.bin     getColor / getFloat of every texture at each point
 *   kat     out.bin                          engine / math known-answer vectors
 *   hdr     in.hdr out_rgba.bin out_rewritten.hdr   reference HDR read + writeHDR
 *   writehdr w h rgba.bin out.hdr            reference MutableImage::writeHDR
 *   matrix  in.bin out.bin                   Matrix::rotate / invert / concat
 */
#include "path-trace.h"
#include "image.h"
#include "image_texture.h"
#include "transform_texture.h"
#include "filter_texture.h"

#include "../include/pt/pt_engine.h"
#include "scene_text.h"

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <fstream>
#include <limits>
#include <map>
#include <thread>

using namespace PathTrace;

namespace
{

/* Test instrument: a Texture whose colour is its lookup coordinate.  Pins the
 * coordinate maps of MirrorBall/Spherical/Transformed textures exactly. */
class CoordTexture : public Texture
{
public:
    virtual Color getColor(Vector3D v) const { return v; }
    virtual Texture *duplicate() const { return new CoordTexture(); }
};

/* Instrument: counts root init() calls (= ray queries). */
class CountingIterator : public SpanIterator
{
public:
    SpanIterator *inner;
    unsigned long long queries = 0;
    explicit CountingIterator(SpanIterator *in) : inner(in) {}
    ~CountingIterator() { delete inner; }
    virtual const Span &operator*() const { return **inner; }
    virtual const Span *operator->() const { return &**inner; }
    virtual bool isAtEnd() const { return inner->isAtEnd(); }
    virtual void next() { inner->next(); }
    virtual void init(const Ray &ray)
    {
        queries++;
        inner->init(ray);
    }
};

std::vector<char> read_file(const std::string &p)
{
    std::ifstream f(p, std::ios::binary);
    if (!f)
        throw std::runtime_error("cannot open " + p);
    return std::vector<char>((std::istreambuf_iterator<char>(f)), std::istreambuf_iterator<char>());
}

struct World
{
    std::map<int, Image> images;
    std::map<int, const Material *> mats;
    std::map<const Material *, int> mat_ids;
    Object *root = nullptr;
};

Matrix mat12(const std::vector<float> &f, size_t o)
{
    return Matrix(f[o + 0], f[o + 1], f[o + 2], f[o + 3], f[o + 4], f[o + 5], f[o + 6], f[o + 7], f[o + 8],
                  f[o + 9], f[o + 10], f[o + 11]);
}

Texture *build_tex(const scenetext::Desc &d, World &w, int id)
{
    const scenetext::Item &t = scenetext::find(d.textures, id, "texture");
    const std::string &ty = t.type;
    auto img = [&](int k) { return w.images.at(t.i[k]); };
    if (ty == "color")
        return new ColorTexture(t.f[0], t.f[1], t.f[2]);
    if (ty == "image")
        return new ImageTexture(img(0));
    if (ty == "image_alpha")
        return new ImageAlphaTexture(img(0));
    if (ty == "skybox")
        return new ImageSkyboxTexture(img(0), img(1), img(2), img(3), img(4), img(5));
    if (ty == "skybox_alpha")
        return new ImageSkyboxAlphaTexture(img(0), img(1), img(2), img(3), img(4), img(5));
    if (ty == "multiply")
        return new MultiplyTexture(Color(t.f[0], t.f[1], t.f[2]), build_tex(d, w, t.i[0]));
    if (ty == "log")
        return new LogTexture(build_tex(d, w, t.i[0]));
    if (ty == "mirrorball")
        return new MirrorBallSkymapTexture(build_tex(d, w, t.i[0]));
    if (ty == "spherical")
        return new SphericalCoordinatesSkymapTexture(build_tex(d, w, t.i[0]));
    if (ty == "xform")
        return new TransformedTexture(mat12(t.f, 0), build_tex(d, w, t.i[0]));
    if (ty == "coord")
        return new CoordTexture();
    throw std::runtime_error("unknown texture " + ty);
}

Object *build_obj(const scenetext::Desc &d, World &w, int id)
{
    const scenetext::Item &o = scenetext::find(d.objects, id, "object");
    const std::string &ty = o.type;
    if (ty == "sphere")
        return new Sphere(Vector3D(o.f[0], o.f[1], o.f[2]), o.f[3], w.mats.at(o.i[0]));
    if (ty == "plane")
        return new Plane(Vector3D(o.f[0], o.f[1], o.f[2]), o.f[3], w.mats.at(o.i[0]));
    if (ty == "union")
        return new Union(build_obj(d, w, o.i[0]), build_obj(d, w, o.i[1]));
    if (ty == "intersection")
        return new Intersection(build_obj(d, w, o.i[0]), build_obj(d, w, o.i[1]));
    if (ty == "difference")
        return new Difference(build_obj(d, w, o.i[0]), build_obj(d, w, o.i[1]));
    if (ty == "xform")
        return new TransformedObject(mat12(o.f, 0), build_obj(d, w, o.i[0]));
    throw std::runtime_error("unknown object " + ty);
}

void build_world(const scenetext::Desc &d, World &w)
{
    for (const scenetext::Item &im : d.images) {
        if (im.type == "hdr") {
            w.images[im.id] = Image(im.path);
        } else {
            int iw = im.i[0], ih = im.i[1];
            std::vector<char> raw = read_file(im.path);
            if (raw.size() != (size_t)iw * ih * 16)
                throw std::runtime_error("raw image size mismatch");
            const float *px = (const float *)raw.data();
            MutableImage mi(iw, ih);
            for (int y = 0; y < ih; y++)
                for (int x = 0; x < iw; x++) {
                    const float *p = px + 4 * ((size_t)y * iw + x);
                    mi.setPixel(x, y, Color(p[0], p[1], p[2]), p[3]);
                }
            w.images[im.id] = (Image)mi;
        }
    }
    for (const scenetext::Item &m : d.materials) {
        Material *mat = new Material(build_tex(d, w, m.i[0]), build_tex(d, w, m.i[1]), build_tex(d, w, m.i[2]),
                                     build_tex(d, w, m.i[3]), m.f[0], build_tex(d, w, m.i[4]));
        w.mats[m.id] = mat;
        w.mat_ids[mat] = m.id;
    }
    w.root = build_obj(d, w, d.root);
}

void write_file(const std::string &p, const void *data, size_t n)
{
    std::ofstream f(p, std::ios::binary);
    f.write((const char *)data, n);
    if (!f)
        throw std::runtime_error("cannot write " + p);
}

int mode_render(int argc, char **argv)
{
    if (argc != 15) {
        fprintf(stderr, "render: bad args\n");
        return 2;
    }
    std::vector<char> txt = read_file(argv[2]);
    scenetext::Desc d = scenetext::parse(std::string(txt.data(), txt.size()));
    World w;
    build_world(d, w);
    int W = atoi(argv[3]), H = atoi(argv[4]), spp = atoi(argv[5]), depth = atoi(argv[6]);
    float sw = scenetext::parse_float(argv[7]), sh = scenetext::parse_float(argv[8]),
          dist = scenetext::parse_float(argv[9]);
    unsigned long long seed = strtoull(argv[10], nullptr, 0);
    std::vector<int> pixels;
    if (std::string(argv[11]) == "all") {
        for (int i = 0; i < W * H; i++) pixels.push_back(i);
    } else {
        std::vector<char> raw = read_file(argv[11]);
        pixels.assign((const int *)raw.data(), (const int *)raw.data() + raw.size() / 4);
    }
    int threads = atoi(argv[12]);
    bool per_sample = atoi(argv[13]) != 0;
    std::string out = argv[14];
    size_t np = pixels.size();
    std::vector<float> result(per_sample ? np * (size_t)spp * 3 : np * 3);
    std::atomic<unsigned long long> queries(0);
    /* The pool deals (pixel, 32-sample block) units, not whole pixels: one
     * pixel's 1024 samples on one thread made a bounded sample's few expensive
     * pixels its tail.  Each unit keeps its samples' colours; a
     * pixel's mean is then tracePixel's own sequential sum over them, so the
     * bits are unchanged.  Pixels go in windows whose per-sample colours fit
     * 256 MB. */
    const int kBlock = 32;
    const size_t nb = ((size_t)spp + kBlock - 1) / kBlock;
    const size_t win = per_sample ? std::max<size_t>(np, 1)
                                  : std::max<size_t>(1, ((size_t)256 << 20) / ((size_t)spp * 12));
    std::vector<float> vals(per_sample ? 0 : std::min(win, np) * (size_t)spp * 3);
    auto t0 = std::chrono::steady_clock::now();
    for (size_t w0 = 0; w0 < np; w0 += win) {
        const size_t wn = std::min(win, np - w0);
        float *vb = per_sample ? &result[w0 * (size_t)spp * 3] : vals.data();
        std::atomic<size_t> next(0);
        auto worker = [&]() {
            CountingIterator it(w.root->makeSpanIterator());
            for (;;) {
                const size_t u = next.fetch_add(1);
                if (u >= wn * nb)
                    break;
                const size_t k = u / nb;
                const int b = (int)(u % nb);
                const int p = pixels[w0 + k], px = p % W, py = p / W;
                for (int s = b * kBlock; s < spp && s < (b + 1) * kBlock; s++) {
                    PtSampleEngine e((uint64_t)seed, (uint64_t)p, (uint64_t)s);
                    Color c = tracePixel(it, px, py, W, H, 1, depth, sw, sh, dist, e);
                    float *o = &vb[(k * spp + s) * 3];
                    o[0] = c.x;
                    o[1] = c.y;
                    o[2] = c.z;
                }
            }
            queries += it.queries;
        };
        std::vector<std::thread> pool;
        for (int t = 0; t < threads; t++) pool.emplace_back(worker);
        for (auto &t : pool) t.join();
        if (!per_sample)
            for (size_t k = 0; k < wn; k++) { /* tracePixel's spp loop: acc += c in sample order, / spp */
                Color acc(0, 0, 0);
                for (int s = 0; s < spp; s++) {
                    const float *v = &vb[(k * spp + s) * 3];
                    acc += Color(v[0], v[1], v[2]);
                }
                acc /= spp;
                result[(w0 + k) * 3 + 0] = acc.x;
                result[(w0 + k) * 3 + 1] = acc.y;
                result[(w0 + k) * 3 + 2] = acc.z;
            }
    }
    double secs = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    write_file(out, result.data(), result.size() * 4);
    printf("{\"seconds\": %.6f, \"samples\": %zu, \"queries\": %llu, \"threads\": %d}\n", secs, np * (size_t)spp,
           (unsigned long long)queries, threads);
    return 0;
}

int mode_rays(int argc, char **argv)
{
    if (argc != 9) {
        fprintf(stderr, "rays: bad args\n");
        return 2;
    }
    std::vector<char> txt = read_file(argv[2]);
    scenetext::Desc d = scenetext::parse(std::string(txt.data(), txt.size()));
    World w;
    build_world(d, w);
    std::vector<char> raw = read_file(argv[3]);
    const float *r = (const float *)raw.data();
    const size_t n = raw.size() / 28;
    const int spp = atoi(argv[4]), depth = atoi(argv[5]), threads = atoi(argv[7]);
    const unsigned long long seed = strtoull(argv[6], nullptr, 0);
    std::vector<float> result(n * 3);
    std::atomic<size_t> next(0);
    auto worker = [&]() {
        std::unique_ptr<SpanIterator> it(w.root->makeSpanIterator());
        for (;;) {
            size_t k = next.fetch_add(1);
            if (k >= n)
                break;
            const float *q = r + 7 * k;
            Ray ray(Vector3D(q[0], q[1], q[2]), Vector3D(q[3], q[4], q[5]));
            Color acc(0, 0, 0);
            for (int s = 0; s < spp; s++) {
                PtSampleEngine e((uint64_t)seed, (uint64_t)k, (uint64_t)s);
                Color c = Color(0, 0, 0);
                c += traceRay(ray, *it, depth, e, q[6]);
                c /= 1;
                acc += c;
            }
            acc /= spp;
            result[3 * k] = acc.x, result[3 * k + 1] = acc.y, result[3 * k + 2] = acc.z;
        }
    };
    std::vector<std::thread> pool;
    for (int t = 0; t < threads; t++) pool.emplace_back(worker);
    for (auto &t : pool) t.join();
    write_file(argv[8], result.data(), result.size() * 4);
    return 0;
}

/* spans: rays.bin = n * 6 floats (origin, dir).  out.bin per ray: int32 count,
 * then count * (start, sN.xyz, sMat, end, eN.xyz, eMat) as 10 x 4 bytes. */
int mode_spans(int argc, char **argv)
{
    if (argc != 5)
        return 2;
    std::vector<char> txt = read_file(argv[2]);
    scenetext::Desc d = scenetext::parse(std::string(txt.data(), txt.size()));
    World w;
    build_world(d, w);
    std::vector<char> raw = read_file(argv[3]);
    const float *r = (const float *)raw.data();
    size_t n = raw.size() / 24;
    std::vector<char> out;
    auto put = [&](const void *p, size_t k) { out.insert(out.end(), (const char *)p, (const char *)p + k); };
    SpanIterator *it = w.root->makeSpanIterator();
    for (size_t k = 0; k < n; k++) {
        Ray ray(Vector3D(r[6 * k], r[6 * k + 1], r[6 * k + 2]), Vector3D(r[6 * k + 3], r[6 * k + 4], r[6 * k + 5]));
        std::vector<Span> spans;
        for (it->init(ray); *it; (*it)++) {
            spans.push_back(**it);
            if (spans.size() > 4096)
                throw std::runtime_error("runaway span list");
        }
        int32_t c = (int32_t)spans.size();
        put(&c, 4);
        for (const Span &s : spans) {
            int32_t sm = s.startMaterial ? w.mat_ids.at(s.startMaterial) : -1;
            int32_t em = s.endMaterial ? w.mat_ids.at(s.endMaterial) : -1;
            float v[8] = {s.start, s.startNormal.x, s.startNormal.y, s.startNormal.z,
                          s.end,   s.endNormal.x,   s.endNormal.y,   s.endNormal.z};
            put(&v[0], 16);
            put(&sm, 4);
            put(&v[4], 16);
            put(&em, 4);
        }
    }
    delete it;
    write_file(argv[4], out.data(), out.size());
    return 0;
}

/* kat: engine and vector-math known answers, written as a flat float/uint
 * stream whose layout tests/test_oracle_golden.py mirrors. */
int mode_kat(int argc, char **argv)
{
    if (argc != 3)
        return 2;
    std::vector<uint32_t> o;
    auto pf = [&](float f) {
        uint32_t u;
        memcpy(&u, &f, 4);
        o.push_back(u);
    };
    // 1. DefaultRandomEngine, seeds 0, 1, 12345: first 5 outputs
    unsigned seeds[3] = {0, 1, 12345};
    for (unsigned s : seeds) {
        DefaultRandomEngine e;
        e.seed(s);
        for (int k = 0; k < 5; k++) o.push_back(e());
    }
    // 2. PtSampleEngine (seed 0x5EED, pixel 7, sample 3): 16 outputs
    {
        PtSampleEngine e(0x5EEDull, 7, 3);
        for (int k = 0; k < 16; k++) o.push_back(e());
    }
    // 3. uniform_real_distribution<float>(0,1) and (-1,1) on DefaultRandomEngine seed 0
    {
        DefaultRandomEngine e;
        uniform_real_distribution<float> u01(0, 1), u11(-1, 1);
        for (int k = 0; k < 4; k++) pf(u01(e));
        for (int k = 0; k < 4; k++) pf(u11(e));
    }
    // 4. Vector3D::rand(e, 1, 0) on PtSampleEngine(0x5EED, 1, 1): 64 draws
    {
        PtSampleEngine e(0x5EEDull, 1, 1);
        for (int k = 0; k < 64; k++) {
            Vector3D v = Vector3D::rand(e, 1, 0);
            pf(v.x);
            pf(v.y);
            pf(v.z);
        }
    }
    // 5. refract / refractStrength / reflect / normalize on a deterministic grid
    {
        PtSampleEngine e(0x5EEDull, 2, 2);
        uniform_real_distribution<float> u(-2, 2);
        for (int k = 0; k < 256; k++) {
            float v[7];
            for (int j = 0; j < 7; j++) v[j] = u(e); /* explicit draw order */
            Vector3D d(v[0], v[1], v[2]), n(v[3], v[4], v[5]);
            float ior = 0.25f + (v[6] + 2) * 0.5f;
            if (k % 17 == 0)
                d = Vector3D(0.3f, 0, -1), n = Vector3D(0, 0, 1), ior = 1 / 1.3f;
            Vector3D r = d.refract(ior, n), rf = d.reflect(n), nn = normalize(d);
            float rs = d.refractStrength(ior, n);
            for (float f : {d.x, d.y, d.z, n.x, n.y, n.z, ior, r.x, r.y, r.z, rs, rf.x, rf.y, rf.z, nn.x, nn.y, nn.z})
                pf(f);
        }
    }
    write_file(argv[2], o.data(), o.size() * 4);
    return 0;
}

int mode_hdr(int argc, char **argv)
{
    if (argc != 5)
        return 2;
    Image img(argv[2]);
    MutableImage mi(img);
    std::vector<float> px((size_t)mi.width() * mi.height() * 4);
    for (unsigned y = 0; y < mi.height(); y++)
        for (unsigned x = 0; x < mi.width(); x++) {
            Color c = mi.getPixel(x, y);
            float *p = &px[4 * ((size_t)y * mi.width() + x)];
            p[0] = c.x;
            p[1] = c.y;
            p[2] = c.z;
            p[3] = img.getPixelAlpha(x, y);
        }
    write_file(argv[3], px.data(), px.size() * 4);
    mi.writeHDR(argv[4]);
    printf("{\"w\": %u, \"h\": %u}\n", mi.width(), mi.height());
    return 0;
}

int mode_writehdr(int argc, char **argv)
{
    if (argc != 6)
        return 2;
    int w = atoi(argv[2]), h = atoi(argv[3]);
    std::vector<char> raw = read_file(argv[4]);
    const float *p = (const float *)raw.data();
    MutableImage mi(w, h);
    for (int y = 0; y < h; y++)
        for (int x = 0; x < w; x++) {
            const float *q = p + 3 * ((size_t)y * w + x);
            mi.setPixel(x, y, Color(q[0], q[1], q[2]));
        }
    mi.writeHDR(argv[5]);
    return 0;
}

/* tex: Texture::getColor and Texture::getFloat (include/texture.h:13-18, through
 * the virtuals, so every subclass's override) of each texture of the scene
 * text, in file order, at every point of points.bin (3 float32 each); out.bin =
 * per texture, per point, r g b value (float32). */
int mode_tex(int argc, char **argv)
{
    if (argc != 5)
        return 2;
    std::vector<char> txt = read_file(argv[2]);
    scenetext::Desc d = scenetext::parse(std::string(txt.data(), txt.size()));
    World w;
    build_world(d, w);
    std::vector<char> raw = read_file(argv[3]);
    const float *p = (const float *)raw.data();
    const size_t n = raw.size() / 12;
    std::vector<float> out;
    for (const scenetext::Item &t : d.textures) {
        Texture *tex = build_tex(d, w, t.id);
        for (size_t k = 0; k < n; k++) {
            const Vector3D v(p[3 * k], p[3 * k + 1], p[3 * k + 2]);
            const Color c = tex->getColor(v);
            out.push_back(c.x), out.push_back(c.y), out.push_back(c.z), out.push_back(tex->getFloat(v));
        }
        delete tex;
    }
    write_file(argv[4], out.data(), out.size() * 4);
    return 0;
}

/* matrix: in.bin = n records of {float axis[3]; float pad; double angle; float m[12]; float m2[12]},
 * out.bin = n records of {rotate(axis, angle)[12], invert(m)[12] (NaN if singular), m.concat(m2)[12]}. */
int mode_matrix(int argc, char **argv)
{
    if (argc != 4)
        return 2;
    std::vector<char> raw = read_file(argv[2]);
    const size_t rec = 4 * 4 + 8 + 48 + 48;
    size_t n = raw.size() / rec;
    std::vector<float> out;
    auto put = [&](const Matrix &m) {
        float v[12] = {m.x00, m.x10, m.x20, m.x30, m.x01, m.x11, m.x21, m.x31, m.x02, m.x12, m.x22, m.x32};
        out.insert(out.end(), v, v + 12);
    };
    for (size_t k = 0; k < n; k++) {
        const char *r = raw.data() + k * rec;
        float axis[3];
        double angle;
        float m[12], m2[12];
        memcpy(axis, r, 12);
        memcpy(&angle, r + 16, 8);
        memcpy(m, r + 24, 48);
        memcpy(m2, r + 72, 48);
        std::vector<float> mv(m, m + 12), m2v(m2, m2 + 12);
        put(Matrix::rotate(Vector3D(axis[0], axis[1], axis[2]), angle));
        try {
            put(invert(mat12(mv, 0)));
        } catch (std::domain_error &) {
            float nan = std::numeric_limits<float>::quiet_NaN();
            for (int j = 0; j < 12; j++) out.push_back(nan);
        }
        put(mat12(mv, 0).concat(mat12(m2v, 0)));
    }
    write_file(argv[3], out.data(), out.size() * 4);
    return 0;
}

} // namespace

int main(int argc, char **argv)
{
    try {
        if (argc < 2)
            return 2;
        std::string m = argv[1];
        if (m == "render")
            return mode_render(argc, argv);
        if (m == "spans")
            return mode_spans(argc, argv);
        if (m == "rays")
            return mode_rays(argc, argv);
        if (m == "kat")
            return mode_kat(argc, argv);
        if (m == "hdr")
            return mode_hdr(argc, argv);
        if (m == "writehdr")
            return mode_writehdr(argc, argv);
        if (m == "matrix")
            return mode_matrix(argc, argv);
        if (m == "tex")
            return mode_tex(argc, argv);
        fprintf(stderr, "unknown mode %s\n", m.c_str());
        return 2;
    } catch (std::exception &e) {
        fprintf(stderr, "ptref error: %s\n", e.what());
        return 1;
    }
}
