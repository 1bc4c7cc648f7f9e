// Builds the north-star scene P1 (pathtrace/scenes.py scene_p1) with the C++
// facade include/pt/PathTrace.hpp, written the way the reference's demo
// builds its world (src/test.cpp:107-145), then
//   facade_p1 key DEPTH                 -> prints the scene's code-object key (no GPU)
//   facade_p1 render W H SPP DEPTH OUT  -> renders on device 0, writes W*H*3 f32 to OUT
//   facade_p1 errors                    -> checks the error mapping (no GPU)
//   facade_p1 spans RAYS OUT            -> world->makeSpanIterator() over each ray of RAYS
//                                          (n x 6 f32): per ray a count, then per span
//                                          t0 n0 m0 t1 n1 m1 (m = material index below)
//   facade_p1 tex HDR PTS OUT           -> getColor / getFloat of MirrorBall(Image(HDR))
//                                          and of a user-defined Texture at each point
//   facade_p1 traceray RAYS DEPTH SPP OUT  -> traceRay for n x 7 caller rays (reference order)
//   facade_p1 latency W H SPP DEPTH THREADS OUT.json -> per-call tracePixel latency,
//                                          one-batch and PixelBatcher throughput
#include <cstdio>
#include <cstdlib>
#include <cmath>
#include <cstring>
#include <chrono>
#include <memory>
#include <thread>
#include <vector>

#include "pt/PathTrace.hpp"

using namespace PathTrace;

/* a reference-style user texture: overrides getColor only (texture.h:13) */
class Checker : public Texture
{
public:
    Color getColor(Vector3D p) const override
    {
        return ((int)std::floor(p.x) + (int)std::floor(p.y) + (int)std::floor(p.z)) % 2 ? Color(1) : Color(0.25f);
    }
    Texture *duplicate() const override { return new Checker; }
};

static std::vector<float> read_f32(const char *path)
{
    std::vector<float> v;
    FILE *f = fopen(path, "rb");
    if (!f)
        return v;
    float x;
    while (fread(&x, 4, 1, f) == 1) v.push_back(x);
    fclose(f);
    return v;
}

/* A user-defined Texture subclass as the reference's API allows (include/
 * texture.h:10-27): a 3-D checkerboard.  getColor runs the body on the host;
 * deviceGetColor hands the same text to the device (pt_tex_device). */
namespace user
{
struct V3
{
    float x, y, z;
};
inline V3 mk(float x, float y, float z)
{
    V3 r;
    r.x = x, r.y = y, r.z = z;
    return r;
}
#define PT_TEXT_(...) #__VA_ARGS__
#define PT_TEXT(...) PT_TEXT_(__VA_ARGS__) /* expands the body macro, then stringises it */
#define CHECKER_BODY                                                                  \
    const float s = prm[0];                                                           \
    const float k = floorf(p.x * s) + floorf(p.y * s) + floorf(p.z * s);              \
    const float odd = k - 2.0f * floorf(k * 0.5f);                                    \
    return odd != 0.0f ? mk(prm[1], prm[2], prm[3]) : mk(prm[4], prm[5], prm[6]);
inline V3 checker(V3 p, const float *prm) { CHECKER_BODY }
} // namespace user

class CheckerTexture : public Texture
{
public:
    explicit CheckerTexture(const std::vector<float> &prm) : prm_(prm) {}
    Color getColor(Vector3D pos) const override
    {
        const user::V3 c = user::checker(user::mk(pos.x, pos.y, pos.z), prm_.data());
        return Color(c.x, c.y, c.z);
    }
    Texture *duplicate() const override { return new CheckerTexture(prm_); }
    const char *deviceGetColor() const override { return PT_TEXT(CHECKER_BODY); }
    std::vector<float> deviceParams() const override { return prm_; }

private:
    std::vector<float> prm_;
};

/* A user-defined Object subclass (include/object.h:10-24) with the
 * reference sphere's arithmetic (src/sphere.cpp:31-49) as its device form:
 * P1 built with it in place of one of its spheres renders P1's frame. */
class UserSphere : public Object
{
public:
    UserSphere(Vector3D c, float r, const Material *m) : c_(c), r_(r), m_(m) {}
    Object *duplicate() const override { return new UserSphere(c_, r_, m_); }
    const char *deviceSpan() const override
    {
        return "const V3 oc = mk(o.x - prm[0], o.y - prm[1], o.z - prm[2]);"
               "const float a = dot(d, d), b = dot(oc, d), c = dot(oc, oc) - prm[3];"
               "const float disc = b * b - a * c;"
               "if (disc <= 1e-3f) return false;"
               "const float s = sqrtf(disc);"
               "t0 = (-b - s) / a; t1 = (-b + s) / a; return true;";
    }
    const char *deviceNormal() const override
    {
        return "const V3 q = mk(p.x - prm[0], p.y - prm[1], p.z - prm[2]);"
               "float m = sqrtf(dot(q, q)); if (m == 0.0f) m = 1.0f;"
               "return mk(q.x / m, q.y / m, q.z / m);";
    }
    std::vector<float> deviceParams() const override { return {c_.x, c_.y, c_.z, r_ * r_}; }
    const Material *deviceMaterial() const override { return m_; }

private:
    Vector3D c_;
    float r_;
    const Material *m_;
};

int main(int argc, char **argv)
{
    if (argc < 2)
        return 2;
    Material diffuse(new ColorTexture(0.8f), new ColorTexture(1));
    Material mirror(new ColorTexture(0.99f), new ColorTexture(0));
    Material glass(new ColorTexture(0.7f), new ColorTexture(0), new ColorTexture(0), new ColorTexture(0.9f), 1.3f,
                   new ColorTexture(1));
    Material sky(new ColorTexture(0), new ColorTexture(0), new ColorTexture(0.5f, 0.7f, 1.0f));
    Object *left = new Difference(new Union(new Sphere(Vector3D(-1, 0, -4), .6f, &diffuse),
                                            new Sphere(Vector3D(-.5f, 0, -4), .6f, &diffuse)),
                                  new Sphere(Vector3D(-.7f, .3f, -3.6f), .4f, &diffuse));
    Object *right = new Difference(new Union(new Sphere(Vector3D(1, 0, -4), .6f, &glass),
                                             new Sphere(Vector3D(1.4f, .2f, -4.2f), .5f, &mirror)),
                                   new Sphere(Vector3D(1, 0, -3.4f), .3f, &glass));
    std::unique_ptr<Object> world(new Union(left, new Union(right, new Plane(Vector3D(0, 0, 1), 200, &sky))));

    try {
        if (!strcmp(argv[1], "errors")) {
            bool ok = false;
            try {
                invert(Matrix::scale(0.0f));
            } catch (std::domain_error &) {
                ok = true;
            }
            if (!ok)
                return 3;
            ok = false;
            try {
                Image("/nonexistent.hdr");
            } catch (ImageLoadError &) {
                ok = true;
            }
            if (!ok)
                return 4;
            { /* PixelBatcher: a bad coordinate fails its own caller before it joins a batch (no device work) */
                std::unique_ptr<SpanIterator> it(world->makeSpanIterator());
                PixelBatcher q(*it, 16, 16, 1, 4, 16, 16, 32);
                ok = false;
                try {
                    q.tracePixel(-1, 3);
                } catch (std::invalid_argument &) {
                    ok = true;
                }
                if (!ok || q.launches() != 0)
                    return 5;
            }
            Matrix r = Matrix::rotateY(0.5);
            Matrix id = r.concat(invert(r));
            printf("errors ok %.6f %.6f\n", id.x00, id.x11);
            return 0;
        }
        if (!strcmp(argv[1], "spans") && argc == 4) {
            const Material *mats[4] = {&diffuse, &mirror, &glass, &sky};
            auto mi = [&](const Material *m) {
                for (int k = 0; k < 4; k++)
                    if (mats[k] == m)
                        return k;
                return -1;
            };
            std::vector<float> rays = read_f32(argv[2]);
            std::unique_ptr<SpanIterator> it(world->makeSpanIterator());
            FILE *f = fopen(argv[3], "wb");
            if (!f)
                return 5;
            for (size_t r = 0; r + 6 <= rays.size(); r += 6) {
                it->init(Ray(Vector3D(rays[r], rays[r + 1], rays[r + 2]), Vector3D(rays[r + 3], rays[r + 4], rays[r + 5])));
                std::vector<float> rec;
                int32_t count = 0;
                for (; !it->isAtEnd(); it->next(), count++) {
                    const Span &sp = **it;
                    int32_t m0 = mi(sp.startMaterial), m1 = mi(sp.endMaterial);
                    float a[4] = {sp.start, sp.startNormal.x, sp.startNormal.y, sp.startNormal.z};
                    float b[4] = {sp.end, sp.endNormal.x, sp.endNormal.y, sp.endNormal.z};
                    float m0f, m1f;
                    memcpy(&m0f, &m0, 4), memcpy(&m1f, &m1, 4);
                    rec.insert(rec.end(), a, a + 4), rec.push_back(m0f);
                    rec.insert(rec.end(), b, b + 4), rec.push_back(m1f);
                }
                fwrite(&count, 4, 1, f);
                fwrite(rec.data(), 4, rec.size(), f);
            }
            fclose(f);
            return 0;
        }
        if (!strcmp(argv[1], "tex") && argc == 5) {
            std::unique_ptr<Texture> mb(new MirrorBallSkymapTexture(new ImageTexture(Image(argv[2]))));
            Checker user;
            std::vector<float> pts = read_f32(argv[3]);
            FILE *f = fopen(argv[4], "wb");
            if (!f)
                return 5;
            const size_t n = pts.size() / 3;
            std::vector<Vector3D> P;
            for (size_t k = 0; k < n; k++) P.push_back(Vector3D(pts[3 * k], pts[3 * k + 1], pts[3 * k + 2]));
            std::vector<Color> C(n);
            std::vector<float> V(n);
            mb->getColors(P.data(), n, C.data(), V.data()); /* one device call for all points */
            for (size_t k = 0; k < n; k++) {
                if (k < 4) { /* the per-point virtuals give the same bits */
                    Color c = mb->getColor(P[k]);
                    float v = mb->getFloat(P[k]);
                    if (memcmp(&c, &C[k], sizeof c) || memcmp(&v, &V[k], 4))
                        return 6;
                }
                Color u = user.getColor(P[k]);
                float rec[8] = {C[k].x, C[k].y, C[k].z, V[k], u.x, u.y, u.z, user.getFloat(P[k])};
                fwrite(rec, 4, 8, f);
            }
            fclose(f);
            return 0;
        }
        if (!strcmp(argv[1], "tracepixel") && argc == 7) {
            /* the reference demo's per-pixel call (src/test.cpp:450, 503) */
            const int W = atoi(argv[2]), H = atoi(argv[3]), spp = atoi(argv[4]), depth = atoi(argv[5]);
            std::unique_ptr<SpanIterator> spanIterator(world->makeSpanIterator());
            std::vector<Color> img;
            FrameEngine engine; /* run seed 0x5EED, fast order: Renderer::render's defaults */
            for (int y = 0; y < H; y++)
                for (int x = 0; x < W; x++)
                    img.push_back(tracePixel(*spanIterator, x, y, W, H, spp, depth, (float)W, (float)H,
                                             (float)(2 * (W < H ? W : H)), engine));
            /* the demo's exact call shape (global engine, int screen sizes) and
             * a block corner one past the right edge: they run */
            const int ScreenWidth = W, ScreenHeight = H;
            Color c = tracePixel(*spanIterator, W, 0, ScreenWidth, ScreenHeight, spp, depth, ScreenWidth,
                                 ScreenHeight, (ScreenWidth < ScreenHeight ? ScreenWidth : ScreenHeight) * 2);
            if (!(c.x == c.x))
                return 7;
            /* the engine-less overload is the global FrameEngine's (run seed
             * 0x5EED, fast order): Renderer::render's pixel */
            Color g = tracePixel(*spanIterator, 3 % W, 1 % H, ScreenWidth, ScreenHeight, spp, depth, ScreenWidth,
                                 ScreenHeight, (ScreenWidth < ScreenHeight ? ScreenWidth : ScreenHeight) * 2);
            if (memcmp(&g, &img[(size_t)(1 % H) * W + 3 % W], sizeof(Color)))
                return 15;
            /* a reference-style engine T: two of its draws (high word first)
             * are the call's run seed -- the same bits as a FrameEngine of that seed */
            struct Lcg /* the reference's DefaultRandomEngine recurrence, include/path-trace.h:21-54 */
            {
                uint64_t v = 0x12476242;
                static unsigned min() { return 0; }
                static unsigned max() { return 0xFFFFFFFF; }
                unsigned operator()() { return (unsigned)((v = 214013 * v + 2531011) >> 32); }
            } lcg, twin;
            Color t = tracePixel(*spanIterator, 2 % W, 2 % H, W, H, spp, depth, (float)W, (float)H,
                                 (float)(2 * (W < H ? W : H)), lcg);
            const uint64_t hi = twin(), lo = twin();
            FrameEngine seeded((hi << 32) | lo);
            Color u = tracePixel(*spanIterator, 2 % W, 2 % H, W, H, spp, depth, (float)W, (float)H,
                                 (float)(2 * (W < H ? W : H)), seeded);
            if (memcmp(&t, &u, sizeof(Color)) || lcg.v != twin.v)
                return 16;
            /* ... and successive calls draw fresh run seeds, as the reference's
             * shared engine hands successive calls fresh numbers */
            Color t2 = tracePixel(*spanIterator, 2 % W, 2 % H, W, H, spp, depth, (float)W, (float)H,
                                  (float)(2 * (W < H ? W : H)), lcg);
            if (lcg.v == twin.v || !(t2.x == t2.x))
                return 17;
            /* a batch that holds the block corners x == W of every row: the
             * in-frame pixels keep their bits (keys never depend on the batch) */
            std::vector<int32_t> bx, by;
            for (int y = 0; y < H; y++)
                for (int x = 0; x <= W; x++) bx.push_back(x), by.push_back(y);
            std::vector<Color> batch(bx.size());
            tracePixels(*spanIterator, bx.data(), by.data(), bx.size(), batch.data(), W, H, spp, depth, (float)W,
                        (float)H, (float)(2 * (W < H ? W : H)), engine);
            for (int y = 0; y < H; y++) {
                for (int x = 0; x < W; x++)
                    if (memcmp(&batch[(size_t)y * (W + 1) + x], &img[(size_t)y * W + x], sizeof(Color)))
                        return 8;
                /* the corner (W, y) alone gives the bits it had in the batch */
                Color e = tracePixel(*spanIterator, W, y, W, H, spp, depth, (float)W, (float)H,
                                     (float)(2 * (W < H ? W : H)), engine);
                if (memcmp(&e, &batch[(size_t)y * (W + 1) + W], sizeof(Color)))
                    return 9;
            }
            FILE *f = fopen(argv[6], "wb");
            if (!f)
                return 5;
            fwrite(img.data(), sizeof(Color), img.size(), f);
            fclose(f);
            return 0;
        }
        if (!strcmp(argv[1], "traceray") && argc == 6) {
            /* traceRay for caller rays (RAYS: n x 7 floats) in reference order:
             * the batch with `spp` samples per ray goes to OUT; per-call traceRay,
             * the T-engine overload and the float-coordinate tracePixel are
             * checked against batches with the same keys */
            std::vector<float> rv = read_f32(argv[2]);
            const int depth = atoi(argv[3]), spp = atoi(argv[4]);
            const size_t n = rv.size() / 7;
            std::vector<Ray> rays;
            std::vector<float> str;
            for (size_t k = 0; k < n; k++) {
                const float *q = &rv[7 * k];
                rays.push_back(Ray(Vector3D(q[0], q[1], q[2]), Vector3D(q[3], q[4], q[5])));
                str.push_back(q[6]);
            }
            std::unique_ptr<SpanIterator> it(world->makeSpanIterator());
            std::vector<Color> batch(n), one(n), calls(n);
            FrameEngine eb(0x5EED, PT_ORDER_REFERENCE);
            traceRays(*it, rays.data(), str.data(), n, batch.data(), depth, eb, spp);
            if (eb.rays != n)
                return 10;
            FrameEngine e1(0x5EED, PT_ORDER_REFERENCE), e2(0x5EED, PT_ORDER_REFERENCE);
            traceRays(*it, rays.data(), str.data(), n, one.data(), depth, e1);
            for (size_t k = 0; k < n && k < 24; k++) /* the per-call overload: the engine's next key */
                if (memcmp(&one[k], &(calls[k] = traceRay(rays[k], *it, depth, e2, str[k])), sizeof(Color)))
                    return 11;
            struct Lcg /* a reference-style engine type (include/vector3d.h:14-34) */
            {
                uint64_t v = 0x12476242;
                static unsigned min() { return 0; }
                static unsigned max() { return 0xFFFFFFFF; }
                unsigned operator()() { return (unsigned)((v = 214013 * v + 2531011) >> 32); }
            } lcg;
            Color t = traceRay(rays[0], *it, depth, lcg, 1.0f);
            Color p = tracePixel(*it, 10.5f, 7.25f, 40.0f, 30.0f, 3, depth, 40.0f, 30.0f, 60.0f, lcg);
            if (!(t.x == t.x) || !(p.x == p.x))
                return 12;
            /* float tracePixel == the batch of its camera ray (same keys) */
            FrameEngine e3, e4;
            Color fp = tracePixel(*it, 10.5f, 7.25f, 40.0f, 30.0f, 3, depth, 40.0f, 30.0f, 60.0f, e3);
            const float x = 2 * 10.5f / 40.0f - 1, y = 1 - 2 * 7.25f / 30.0f;
            Ray cam(Vector3D(0, 0, 0), Vector3D(x * 40.0f, y * 30.0f, -60.0f));
            Color fb;
            traceRays(*it, &cam, nullptr, 1, &fb, depth, e4, 3);
            if (memcmp(&fp, &fb, sizeof(Color)))
                return 13;
            FILE *f = fopen(argv[5], "wb");
            if (!f)
                return 5;
            fwrite(batch.data(), sizeof(Color), n, f);
            fclose(f);
            return 0;
        }
        if (!strcmp(argv[1], "usertex") && argc == 7) {
            /* P0's shape with the floor's emission a user CheckerTexture (tests/
             * test_user_texture.py CHECKER): the frame, and the host override
             * against the device body at a few points (exit 18 on a mismatch) */
            const int W = atoi(argv[2]), H = atoi(argv[3]), spp = atoi(argv[4]), depth = atoi(argv[5]);
            Material mdiff(new ColorTexture(0.8f), new ColorTexture(1));
            Material mfloor(new ColorTexture(0), new ColorTexture(0),
                            new CheckerTexture({2.0f, 1.0f, 0.9f, 0.3f, 0.2f, 0.3f, 1.0f}));
            std::unique_ptr<Object> w(new Union(new Union(new Sphere(Vector3D(-1, 0, -4), .5f, &mdiff),
                                                          new Sphere(Vector3D(1, 0, -4), .5f, &mirror)),
                                                new Union(new Sphere(Vector3D(0, .3f, -5), .5f, &mdiff),
                                                          new Plane(Vector3D(0, 1, 0), .5f, &mfloor))));
            const Texture *chk = mfloor.emissive;
            const Vector3D pts[4] = {Vector3D(0.1f, 0.2f, 0.3f), Vector3D(-0.6f, 0.7f, 1.4f),
                                     Vector3D(2.5f, -3.5f, 0.25f), Vector3D(-7.25f, -0.5f, -3.0f)};
            Color dev[4];
            float val[4];
            chk->getColors(pts, 4, dev, val);
            for (int k = 0; k < 4; k++) {
                const Color h = chk->getColor(pts[k]);
                if (memcmp(&h, &dev[k], sizeof h))
                    return 18;
            }
            Renderer r(w.get());
            Renderer::Settings st;
            st.width = W, st.height = H, st.sampleCount = spp, st.rayDepth = depth;
            std::vector<Color> img = r.render(st);
            FILE *f = fopen(argv[6], "wb");
            if (!f)
                return 5;
            fwrite(img.data(), sizeof(Color), img.size(), f);
            fclose(f);
            return 0;
        }
        if (!strcmp(argv[1], "latency") && argc == 8) {
            /* the demo's per-pixel call shape against the device: per-call
             * tracePixel latency, one batch for the frame, and the PixelBatcher
             * under THREADS host threads each calling tracePixel pixel by pixel */
            const int W = atoi(argv[2]), H = atoi(argv[3]), spp = atoi(argv[4]), depth = atoi(argv[5]);
            const int threads = atoi(argv[6]);
            const float sw = (float)W, sh = (float)H, dist = (float)(2 * (W < H ? W : H));
            std::unique_ptr<SpanIterator> it(world->makeSpanIterator());
            FrameEngine eng;
            using clk = std::chrono::steady_clock;
            auto secs = [](clk::time_point a) { return std::chrono::duration<double>(clk::now() - a).count(); };
            tracePixel(*it, 0, 0, W, H, spp, depth, sw, sh, dist, eng); /* compile / load / allocate */
            const int ncall = W * H < 256 ? W * H : 256;
            clk::time_point t0 = clk::now();
            for (int k = 0; k < ncall; k++)
                tracePixel(*it, k % W, k / W, W, H, spp, depth, sw, sh, dist, eng);
            const double per_call = secs(t0) / ncall;
            /* per-call breakdown (pt_call_profile), mean over the calls: the top
             * rows above (sky: one query per sample) and pixels spread over the
             * frame (Weyl sequence), plain and with the launches' HIP events */
            double prof[2][2][PT_PROF_N] = {};
            for (int timed = 0; timed < 2; timed++) {
                if (timed)
                    setenv("PT_CALL_KERNEL_TIME", "1", 1);
                for (int spread = 0; spread < 2; spread++)
                    for (int k = 0; k < ncall; k++) {
                        const long long i = spread ? (long long)((k * 0.6180339887 - (long long)(k * 0.6180339887)) *
                                                                 (double)(W * H))
                                                   : k;
                        tracePixel(*it, (int)(i % W), (int)(i / W), W, H, spp, depth, sw, sh, dist, eng);
                        double one[PT_PROF_N];
                        pt_call_profile(one, PT_PROF_N);
                        for (int j = 0; j < PT_PROF_N; j++) prof[timed][spread][j] += one[j] / ncall;
                    }
                unsetenv("PT_CALL_KERNEL_TIME");
            }
            std::vector<int32_t> xs, ys;
            for (int y = 0; y < H; y++)
                for (int x = 0; x < W; x++) xs.push_back(x), ys.push_back(y);
            std::vector<Color> frame(xs.size()), viaq(xs.size());
            t0 = clk::now();
            tracePixels(*it, xs.data(), ys.data(), xs.size(), frame.data(), W, H, spp, depth, sw, sh, dist, eng);
            const double batch = secs(t0);
            uint64_t launches = 0;
            double pooled = 0;
            {
                PixelBatcher q(*it, W, H, spp, depth, sw, sh, dist, eng, 4096, 200);
                t0 = clk::now();
                std::vector<std::thread> pool;
                for (int t = 0; t < threads; t++)
                    pool.emplace_back([&, t] {
                        for (int y = t; y < H; y += threads)
                            for (int x = 0; x < W; x++) viaq[(size_t)y * W + x] = q.tracePixel(x, y);
                    });
                for (auto &th : pool) th.join();
                pooled = secs(t0);
                launches = q.launches();
            }
            if (memcmp(frame.data(), viaq.data(), frame.size() * sizeof(Color)))
                return 14;
            FILE *f = fopen(argv[7], "w");
            if (!f)
                return 5;
            static const char *names[PT_PROF_N] = {"total", "setup", "enqueue", "wait", "d2h", "kernel", "reduce"};
            std::string bd = "{";
            for (int timed = 0; timed < 2; timed++)
                for (int spread = 0; spread < 2; spread++) {
                    char b[96];
                    snprintf(b, sizeof b, "%s\"%s_%s\": {", bd.size() > 1 ? ", " : "", timed ? "events" : "plain",
                             spread ? "spread_pixels" : "top_rows");
                    bd += b;
                    for (int j = 0; j < PT_PROF_N; j++) {
                        if (!timed && j >= PT_PROF_KERNEL)
                            continue;
                        snprintf(b, sizeof b, "%s\"%s\": %.1f", j ? ", " : "", names[j], prof[timed][spread][j]);
                        bd += b;
                    }
                    bd += "}";
                }
            bd += "}";
            fprintf(f, "{\"per_call_breakdown_us\": %s, ", bd.c_str());
            fprintf(f,
                    "\"W\": %d, \"H\": %d, \"spp\": %d, \"depth\": %d, \"threads\": %d, "
                    "\"per_call_us\": %.1f, \"per_call_calls\": %d, \"batch_s\": %.6f, \"batch_us_per_pixel\": %.3f, "
                    "\"batcher_s\": %.6f, \"batcher_launches\": %llu, \"batcher_mean_batch\": %.1f, "
                    "\"batcher_us_per_pixel\": %.3f}\n",
                    W, H, spp, depth, threads, per_call * 1e6, ncall, batch, batch * 1e6 / (W * H), pooled,
                    (unsigned long long)launches, (double)(W * H) / (double)(launches ? launches : 1),
                    pooled * 1e6 / (W * H));
            fclose(f);
            return 0;
        }
        Renderer renderer(world.get());
        if (!strcmp(argv[1], "key") && argc == 3) {
            printf("%s\n", pt_scene_kernel_key(renderer.handle(), atoi(argv[2])));
            return 0;
        }
        if (!strcmp(argv[1], "userobj") && argc == 7) {
            /* P1 with its glass sphere (1, 0, -4) a UserSphere */
            Object *l = new Difference(new Union(new Sphere(Vector3D(-1, 0, -4), .6f, &diffuse),
                                                 new Sphere(Vector3D(-.5f, 0, -4), .6f, &diffuse)),
                                       new Sphere(Vector3D(-.7f, .3f, -3.6f), .4f, &diffuse));
            Object *r = new Difference(new Union(new UserSphere(Vector3D(1, 0, -4), .6f, &glass),
                                                 new Sphere(Vector3D(1.4f, .2f, -4.2f), .5f, &mirror)),
                                       new Sphere(Vector3D(1, 0, -3.4f), .3f, &glass));
            std::unique_ptr<Object> w(new Union(l, new Union(r, new Plane(Vector3D(0, 0, 1), 200, &sky))));
            Renderer ur(w.get());
            Renderer::Settings st;
            st.width = atoi(argv[2]), st.height = atoi(argv[3]);
            st.sampleCount = atoi(argv[4]), st.rayDepth = atoi(argv[5]);
            std::vector<Color> img = ur.render(st);
            FILE *f = fopen(argv[6], "wb");
            if (!f)
                return 5;
            fwrite(img.data(), sizeof(Color), img.size(), f);
            fclose(f);
            return 0;
        }
        if (!strcmp(argv[1], "render") && argc == 7) {
            Renderer::Settings st;
            st.width = atoi(argv[2]), st.height = atoi(argv[3]);
            st.sampleCount = atoi(argv[4]), st.rayDepth = atoi(argv[5]);
            std::vector<Color> img = renderer.render(st);
            FILE *f = fopen(argv[6], "wb");
            if (!f)
                return 5;
            fwrite(img.data(), sizeof(Color), img.size(), f);
            fclose(f);
            return 0;
        }
    } catch (std::exception &e) {
        fprintf(stderr, "facade_p1: %s\n", e.what());
        return 1;
    }
    return 2;
}
