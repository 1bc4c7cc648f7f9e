/*
 * codegen.cpp -- flattens a scene graph into a device module: the CSG tree
 * becomes a compile-time type over pt_device.h's node templates, every float
 * the nodes and textures need goes into the parameter block P at a fixed
 * offset, and the materials become switch dispatchers.  The reference's
 * virtual calls (SpanIterator::init/next, Texture::getColor/getFloat) thus
 * turn into straight-line, fully inlined code per scene.
 */
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <fstream>
#include <sstream>
#include <vector>

#include <cfloat>
#include <cmath>
#include "internal.h"

namespace pt
{

namespace
{

struct Gen
{
    const SceneImpl &s;
    std::vector<float> P;
    std::map<int, int> mat_index;   /* scene material id -> compact index */
    std::vector<int> mats;          /* compact index -> scene material id */
    std::map<int, int> img_slot;    /* scene image id -> slot */
    std::vector<int> images;
    int prim = 0, spheres = 0, planes = 0;
    int depth_guard = 0;
    int xf_depth = 0;          /* TransformedObjects above the node being generated */
    int unit_axis[3] = {0, 0, 0}; /* planes with normal +-e_k outside transforms */
    std::vector<std::pair<size_t, int>> unit_planes; /* (position of the ",U" mark in a node string, axis) */
    std::map<int, int> user_tex; /* User texture id -> offset of its parameters in P */
    std::vector<int> user_obj;   /* User objects reached (their bodies become UObjB_<id>) */

    explicit Gen(const SceneImpl &sc) : s(sc) {}

    /* A bound on |getColor| of texture id over every input point, as the
     * device evaluates it (pt_device.h T* templates), or +inf when none is
     * known (NaN, infinities, user code, TCoord).  Image lookups are
     * bounds-checked (a miss is +0), so an image texture is bounded by its
     * texels whatever point it is asked about; the maps and transforms only
     * move the point; LogTexture's filter lies in (0.1, 1] for finite input. */
    double color_bound(int id, int guard = 0) const
    {
        const double INF = HUGE_VAL;
        if (guard > 64)
            return INF;
        const TexRec &x = s.textures.at(id);
        auto fin = [](double v) { return std::fabs(v) <= (double)FLT_MAX ? std::fabs(v) : HUGE_VAL; };
        auto img = [&](int k) {
            if (k < 0 || k >= (int)s.images.size())
                return 0.0;
            double b = 0.0;
            for (float v : s.images[k].rgba) b = std::max(b, fin(v));
            return b;
        };
        double b = 0.0;
        switch (x.kind) {
        case TexKind::Color:
            for (int c = 0; c < 3; c++) b = std::max(b, fin(x.f[c]));
            return b;
        case TexKind::Image:
        case TexKind::ImageAlpha:
            return img(x.img[0]);
        case TexKind::Skybox:
        case TexKind::SkyboxAlpha:
            for (int k = 0; k < 6; k++) b = std::max(b, img(x.img[k]));
            return b;
        case TexKind::Multiply:
            for (int c = 0; c < 3; c++) b = std::max(b, fin(x.f[c]));
            b *= color_bound(x.child, guard + 1);
            return b <= (double)FLT_MAX ? b : INF; /* a product of finite floats below FLT_MAX rounds finite */
        case TexKind::Log:
            return color_bound(x.child, guard + 1) <= (double)FLT_MAX ? 1.0 : INF;
        case TexKind::MirrorBall:
        case TexKind::Spherical:
        case TexKind::Xform:
            return color_bound(x.child, guard + 1);
        case TexKind::Coord:
        case TexKind::User:
            return INF;
        }
        return INF;
    }

    int put(const float *v, int n)
    {
        int off = (int)P.size();
        P.insert(P.end(), v, v + n);
        return off;
    }

    int material(int id)
    {
        auto it = mat_index.find(id);
        if (it != mat_index.end())
            return it->second;
        int k = (int)mats.size();
        if (k >= 4096)
            throw Error(PT_ERR_ARG, "too many materials (max 4096)");
        mat_index[id] = k;
        mats.push_back(id);
        return k;
    }

    int slot(int img)
    {
        auto it = img_slot.find(img);
        if (it != img_slot.end())
            return it->second;
        int k = (int)images.size();
        img_slot[img] = k;
        images.push_back(img);
        return k;
    }

    std::string obj(int id)
    {
        if (++depth_guard > 10000)
            throw Error(PT_ERR_ARG, "scene graph too deep");
        const ObjRec &o = s.objects.at(id);
        std::ostringstream t;
        switch (o.kind) {
        case ObjKind::Sphere: {
            float v[4] = {o.f[0], o.f[1], o.f[2], o.f[3] * o.f[3]}; /* r_squared = r * r, sphere.cpp:10 */
            int off = put(v, 4);
            t << "Sph<" << prim++ << "," << off << "," << material(o.mat) << ">";
            spheres++;
            break;
        }
        case ObjKind::Plane: {
            int off = put(o.f, 4);
            /* axis-aligned normal: lets the scatter loop's dark test be a sign test */
            int ax = -1, nz = 0;
            for (int k = 0; k < 3; k++)
                if (o.f[k] != 0.0f) {
                    nz++;
                    ax = 2 * k + (o.f[k] < 0.0f ? 1 : 0);
                }
            if (nz != 1 || !std::isfinite(o.f[ax >> 1]))
                ax = -1;
            /* a unit axis normal outside transforms: the plane may share the
             * ray's reciprocal of that direction component with the other
             * such planes of its axis (marked here, decided once the whole
             * tree is known: see shared_axes) */
            const bool unit = ax >= 0 && xf_depth == 0 && std::fabs(o.f[ax >> 1]) == 1.0f;
            t << "Pln<" << prim++ << "," << off << "," << material(o.mat) << "," << ax;
            if (unit) {
                unit_axis[ax >> 1]++;
                t << "@" << (ax >> 1);
            }
            t << ">";
            planes++;
            break;
        }
        case ObjKind::Union:
        case ObjKind::Intersection:
        case ObjKind::Difference: {
            const char *n = o.kind == ObjKind::Union ? "Uni" : o.kind == ObjKind::Intersection ? "Isect" : "Diff";
            std::string a = obj(o.a);
            std::string b = obj(o.b);
            t << n << "<" << a << "," << b << ">";
            break;
        }
        case ObjKind::User: {
            const int off = (int)P.size();
            P.insert(P.end(), o.params.begin(), o.params.end());
            if (std::find(user_obj.begin(), user_obj.end(), id) == user_obj.end())
                user_obj.push_back(id);
            t << "UObj<" << prim++ << "," << off << "," << material(o.mat) << ",UObjB_" << id << ">";
            break;
        }
        case ObjKind::Xform: {
            float inv[12];
            mat_inverse(o.f, inv); /* TransformedSpanIterator: inv(invert(m)), object.h:49-51 */
            int moff = put(o.f, 12);
            int ioff = put(inv, 12);
            xf_depth++;
            const std::string child = obj(o.a);
            xf_depth--;
            t << "Xf<" << moff << "," << ioff << "," << child << ">";
            break;
        }
        }
        if (prim >= (1 << 17))
            throw Error(PT_ERR_ARG, "too many primitives");
        return t.str();
    }

    /* The planes marked '@k' share the ray's reciprocal of component k when
     * at least two of them lie on axis k: the mark becomes the Pln UNIT
     * argument there and disappears elsewhere; mask = the shared axes
     * (PT_AXIS_SHARE). */
    std::string shared_axes(const std::string &t, int &mask) const
    {
        mask = 0;
        for (int k = 0; k < 3; k++)
            if (unit_axis[k] >= 2)
                mask |= 1 << k;
        std::string r;
        r.reserve(t.size());
        for (size_t i = 0; i < t.size(); i++) {
            if (t[i] == '@' && i + 1 < t.size()) {
                if ((mask >> (t[i + 1] - '0')) & 1)
                    r += ",1";
                i++;
            } else {
                r += t[i];
            }
        }
        return r;
    }

    std::string tex(int id)
    {
        const TexRec &x = s.textures.at(id);
        std::ostringstream t;
        switch (x.kind) {
        case TexKind::Color:
            t << "TConst<" << put(x.f, 3) << ">";
            break;
        case TexKind::Coord:
            t << "TCoord";
            break;
        case TexKind::Image:
            t << "TImage<" << slot(x.img[0]) << ">";
            break;
        case TexKind::ImageAlpha:
            t << "TImageAlpha<" << slot(x.img[0]) << ">";
            break;
        case TexKind::Skybox:
        case TexKind::SkyboxAlpha:
            t << (x.kind == TexKind::Skybox ? "TSkybox<" : "TSkyboxAlpha<");
            for (int k = 0; k < 6; k++) t << (k ? "," : "") << slot(x.img[k]);
            t << ">";
            break;
        case TexKind::Multiply: {
            int off = put(x.f, 3);
            t << "TMul<" << off << "," << tex(x.child) << ">";
            break;
        }
        case TexKind::Log:
            t << "TLog<" << tex(x.child) << ">";
            break;
        case TexKind::MirrorBall:
            t << "TMirrorBall<" << tex(x.child) << ">";
            break;
        case TexKind::Spherical:
            t << "TSpherical<" << tex(x.child) << ">";
            break;
        case TexKind::Xform: {
            int off = put(x.f, 12);
            t << "TXf<" << off << "," << tex(x.child) << ">";
            break;
        }
        case TexKind::User:
            if (!user_tex.count(id)) {
                int off = (int)P.size();
                P.insert(P.end(), x.params.begin(), x.params.end());
                user_tex[id] = off;
            }
            t << "UTex_" << id;
            break;
        }
        return t.str();
    }

    /* The user textures' types (pt_tex_device): the caller's bodies see the
     * lookup point `p` and their parameters `prm`; getFloat defaults to the
     * reference's mean of getColor (texture.h:14-18). */
    std::string user_defs() const
    {
        std::ostringstream d;
        for (int id : user_obj) {
            const ObjRec &o = s.objects.at(id);
            d << "struct UObjB_" << id << " {\n"
              << "  __device__ static __forceinline__ bool span(V3 o, V3 d, const float *prm, float &t0, float &t1) {\n"
              << "    (void)prm;\n"
              << "#line 1 \"pt_object_device " << id << " span\"\n"
              << o.span_body << "\n  }\n"
              << "  __device__ static __forceinline__ V3 normal(V3 p, const float *prm) {\n"
              << "    (void)prm;\n"
              << "#line 1 \"pt_object_device " << id << " normal\"\n"
              << o.normal_body << "\n  }\n};\n";
        }
        for (const auto &u : user_tex) {
            const TexRec &x = s.textures.at(u.first);
            d << "struct UTex_" << u.first << " {\n"
              << "  __device__ static __forceinline__ V3 color(V3 p, const Env &e) {\n"
              << "    const float *prm = e.P + " << u.second << ";\n    (void)prm;\n"
              << "#line 1 \"pt_tex_device " << u.first << " getColor\"\n"
              << x.color_body << "\n  }\n"
              << "  __device__ static __forceinline__ float value(V3 p, const Env &e) {\n";
            if (x.value_body.empty()) {
                d << "    return mean3(color(p, e));\n";
            } else {
                d << "    const float *prm = e.P + " << u.second << ";\n    (void)prm;\n"
                  << "#line 1 \"pt_tex_device " << u.first << " getFloat\"\n"
                  << x.value_body << "\n";
            }
            d << "  }\n};\n";
        }
        return d.str();
    }
};

uint64_t fnv1a(const std::string &s, uint64_t h = 1469598103934665603ull)
{
    for (unsigned char c : s) {
        h ^= c;
        h *= 1099511628211ull;
    }
    return h;
}

} // namespace

Generated generate(const SceneImpl &s, int depth, bool rays)
{
    if (s.root < 0)
        throw Error(PT_ERR_ARG, "scene has no root object (pt_set_root)");
    Gen g(s);
    int axis_share = 0;
    const std::string root = g.shared_axes(g.obj(s.root), axis_share);

    /* material dispatchers; texture params are appended after geometry */
    struct MatTypes
    {
        std::string refl, scat, emis, trans, trc;
        bool emis_const;
        int emis_off;
    };
    std::vector<MatTypes> mt;
    for (size_t k = 0; k < g.mats.size(); k++) {
        const MatRec &m = s.materials.at(g.mats[k]);
        MatTypes t;
        t.refl = g.tex(m.reflect);
        t.scat = g.tex(m.scatter);
        t.emis = g.tex(m.emissive);
        t.trans = g.tex(m.transmit);
        t.trc = g.tex(m.trc);
        t.emis_const = s.textures.at(m.emissive).kind == TexKind::Color;
        mt.push_back(t);
    }
    int ior_off = (int)g.P.size();
    for (size_t k = 0; k < g.mats.size(); k++) g.P.push_back(s.materials.at(g.mats[k]).ior);
    bool all_emis_const = true;
    for (auto &t : mt) all_emis_const = all_emis_const && t.emis_const;
    int emis_tab = -1;
    if (all_emis_const) {
        emis_tab = (int)g.P.size();
        for (size_t k = 0; k < g.mats.size(); k++) {
            const TexRec &e = s.textures.at(s.materials.at(g.mats[k]).emissive);
            g.P.insert(g.P.end(), e.f, e.f + 3);
        }
    }

    int maxd = 4;
    while (maxd < depth) maxd *= 2;

    std::ostringstream src;
    /* experiment hook: extra preprocessor definitions, e.g. PT_DEVICE_DEFINES="PT_LEAF_STUB=1" */
    static const bool announce = [] {
        for (const char *h : {"PT_DEVICE_DEFINES", "PT_DEVICE_HEADER"})
            if (const char *v = getenv(h))
                if (*v)
                    fprintf(stderr, "pt: experiment hook %s=\"%s\" active\n", h, v);
        return true;
    }();
    (void)announce;
    if (const char *defs = getenv("PT_DEVICE_DEFINES")) {
        std::istringstream ds(defs);
        std::string d;
        while (ds >> d) {
            size_t eq = d.find('=');
            src << "#define " << (eq == std::string::npos ? d : d.substr(0, eq) + " " + d.substr(eq + 1)) << "\n";
        }
    }
    /* the ray-list module of pt_trace_rays: items are caller rays, not camera samples */
    if (rays)
        src << "#define PT_RAYS 1\n";
    /* per-scene occupancy (pt_scene_set_occupancy): the launch bounds' workgroups per CU */
    if (s.wg_per_cu > 0)
        src << "#define PT_MIN_WAVES " << s.wg_per_cu << "\n";
    /* per-scene spine query form (pt_scene_set_fast_spine) */
    if (s.fast_spine)
        src << "#define PT_FAST_SPINE 1\n";
    /* per-scene lane walk of scatter-free trees (pt_scene_set_lane_walk) */
    if (s.lane_walk > 0)
        src << "#define PT_LANE_WALK " << s.lane_walk << "\n";
    /* per-scene lane walk with scatter loops (pt_scene_set_lane_scatter) */
    if (s.lane_scatter)
        src << "#define PT_LANE_SCATTER 1\n";
    /* Difference-free trees skip a sphere's root and divisions when no lane of
     * the wave meets it (pt_device.h PT_SPHERE_SKIP; same-box A/B,
     * profiles/round4/ab_sphere_skip.txt: C2 +7.2 %, C5 +0.3 %, C3 -10 %) */
    /* ... and run generation rounds of 6 attempts per lane (C2 +1.7 % over 8,
     * 4 of 4 reps on one box, profiles/round4/ab_katt_c2_fixed.txt; 4: -0.9 %;
     * C3 lost 9 % at 6 in round 3) */
    /* axes whose unit-normal planes share the ray's reciprocal (Pln UNIT) */
    if (axis_share)
        src << "#define PT_AXIS_SHARE " << axis_share << "\n";
    if (root.find("Diff<") == std::string::npos)
        src << "#ifndef PT_SPHERE_SKIP\n#define PT_SPHERE_SKIP 1\n#endif\n"
            << "#ifndef PT_KATT\n#define PT_KATT 6\n#endif\n";
    /* trees with a Difference and no lane walks (C3): 10 attempts per lane
     * (+1.1 %, 3 of 3 reps, profiles/round4/ab_katt_c3.txt; 6: -5.4 %), and the
     * next chunk's dequeue in flight while a chunk is traced (round 6, on the
     * final kernel: +0.4 %, 6 of 6 same-box pairs at 1 024 spp,
     * profiles/round6/ab_dequeue_prefetch_c3.txt; round 4's kernel: -0.5 %) */
    else if (s.lane_walk == 0 && !s.lane_scatter)
        src << "#ifndef PT_KATT\n#define PT_KATT 10\n#endif\n"
            << "#ifndef PT_DEQUEUE_PREFETCH\n#define PT_DEQUEUE_PREFETCH 1\n#endif\n";
    /* ... and are scheduled by the iterative max-occupancy strategy (same-box
     * A/B at 1 024 spp: C3 +0.3 %, 4 of 4 reps; C5 -2.6 %, C2 -0.4 %,
     * profiles/round5/ab_sched_maxocc.txt); not when the PT_JIT_OPTIONS hook
     * names a strategy of its own (an LLVM option may occur once) */
    const char *jit_opts = getenv("PT_JIT_OPTIONS");
    const bool maxocc = root.find("Diff<") != std::string::npos && s.lane_walk == 0 && !s.lane_scatter &&
                        !(jit_opts && strstr(jit_opts, "sched-strategy"));
    /* experiment hook: A/B a different device library text in the same run,
     * e.g. PT_DEVICE_HEADER=tools/ab/old.h (profiling only) */
    if (const char *hdr = getenv("PT_DEVICE_HEADER")) {
        std::ifstream f(hdr);
        if (!f)
            throw Error(PT_ERR_ARG, std::string("PT_DEVICE_HEADER not readable: ") + hdr);
        src << f.rdbuf() << "\n";
    } else {
        src << device_library_source() << "\n";
    }
    if (!g.user_obj.empty())
        src << device_user_object_source() << "\n";
    src << "namespace ptgen {\nusing namespace ptd;\n";
    src << g.user_defs();
    src << "typedef " << root << " RootT;\n";
    src << "struct Scene {\n  typedef RootT Root;\n";
    auto dispatch = [&](const char *name, const char *ret, const char *fn, std::string MatTypes::*field) {
        src << "  __device__ static __forceinline__ " << ret << " " << name
            << "(int m, V3 p, const Env &e) {\n    switch (m) {\n";
        for (size_t k = 0; k < mt.size(); k++)
            src << "    case " << k << ": return " << mt[k].*field << "::" << fn << "(p, e);\n";
        src << "    default: return " << (std::string(ret) == "V3" ? "mk(0, 0, 0)" : "0.0f") << ";\n    }\n  }\n";
    };
    /* dark(m): material m's emission is the constant (+0, +0, +0), so a leaf
     * child whose first hit is m (or a miss) contributes weight * +0 */
    src << "  __device__ static constexpr bool dark(int m) { return ";
    std::vector<int> lit_mats;
    for (size_t k = 0; k < g.mats.size(); k++) {
        const TexRec &e = s.textures.at(s.materials.at(g.mats[k]).emissive);
        bool z = e.kind == TexKind::Color;
        for (int c = 0; c < 3 && z; c++) {
            uint32_t bits;
            memcpy(&bits, &e.f[c], 4);
            z = bits == 0u;
        }
        if (!z)
            lit_mats.push_back((int)k);
        src << "m == " << k << " ? " << (z ? "true" : "false") << " : ";
    }
    src << "false; }\n";
    /* emis_finite: every material's emission is finite wherever it is looked
     * up, so a child of weight +-0 adds +-0 (pt_device.h zero_child) */
    bool emis_finite = true;
    for (size_t k = 0; k < g.mats.size() && emis_finite; k++)
        emis_finite = g.color_bound(s.materials.at(g.mats[k]).emissive) <= (double)FLT_MAX;
    src << "  static constexpr bool emis_finite = " << (emis_finite ? "true" : "false") << ";\n";
    if (all_emis_const && lit_mats.size() <= 4) {
        /* few constant emitters: a select chain on scalar-loaded constants
         * (dark materials keep the exact (+0, +0, +0)) instead of a per-lane
         * table load */
        src << "  __device__ static __forceinline__ V3 emis(int m, V3, const Env &e) {\n"
            << "    V3 r = mk(0.0f, 0.0f, 0.0f);\n";
        for (int k : lit_mats)
            src << "    r = m == " << k << " ? mk(e.P[" << emis_tab + 3 * k << "], e.P[" << emis_tab + 3 * k + 1
                << "], e.P[" << emis_tab + 3 * k + 2 << "]) : r;\n";
        src << "    return r;\n  }\n";
    } else if (all_emis_const) {
        src << "  __device__ static __forceinline__ V3 emis(int m, V3, const Env &e) {\n"
            << "    const float *t = e.P + " << emis_tab << " + 3 * m;\n    return mk(t[0], t[1], t[2]);\n  }\n";
    } else {
        dispatch("emis", "V3", "color", &MatTypes::emis);
    }
    dispatch("refl", "V3", "color", &MatTypes::refl);
    dispatch("trans", "V3", "color", &MatTypes::trans);
    dispatch("scat", "float", "value", &MatTypes::scat);
    dispatch("trc", "float", "value", &MatTypes::trc);
    src << "  __device__ static __forceinline__ float ior(int m, const Env &e) { return e.P[" << ior_off
        << " + m]; }\n";
    src << "};\n} // namespace ptgen\n";
    src << "PT_DEFINE_KERNELS(ptgen::Scene, " << maxd << ")\n";

    Generated out;
    out.source = src.str();
    out.params = std::move(g.P);
    if (out.params.empty())
        out.params.push_back(0.0f);
    out.image_ids = g.images;
    out.maxd = maxd;
    if (maxocc)
        out.options = {"-mllvm", "-amdgpu-sched-strategy=iterative-maxocc"};
    out.n_prims = g.prim;
    out.n_spheres = g.spheres;
    out.n_planes = g.planes;
    out.n_mats = (int)g.mats.size();
    out.mat_ids = g.mats;
    char key[40];
    snprintf(key, sizeof key, "%016llx", (unsigned long long)fnv1a(out.source));
    out.key = key;
    return out;
}

Generated generate_query(const SceneImpl &s, int obj, int tex)
{
    Gen g(s);
    std::ostringstream src;
    int axis_share = 0;
    const std::string qroot = obj >= 0 ? g.shared_axes(g.obj(obj), axis_share) : std::string();
    if (axis_share)
        src << "#define PT_AXIS_SHARE " << axis_share << "\n";
    const std::string qtex = tex >= 0 ? g.tex(tex) : std::string();
    src << device_library_source() << "\n";
    if (!g.user_obj.empty())
        src << device_user_object_source() << "\n";
    src << "namespace ptgen {\nusing namespace ptd;\n";
    src << g.user_defs();
    if (obj >= 0)
        src << "typedef " << qroot << " QRoot;\n";
    if (tex >= 0)
        src << "typedef " << qtex << " QTex;\n";
    src << "} // namespace ptgen\n";
    if (obj >= 0)
        src << "PT_DEFINE_QUERY(ptgen::QRoot)\n";
    if (tex >= 0)
        src << "PT_DEFINE_TEXEVAL(ptgen::QTex)\n";
    Generated out;
    out.source = src.str();
    out.params = std::move(g.P);
    if (out.params.empty())
        out.params.push_back(0.0f);
    out.image_ids = g.images;
    out.n_prims = g.prim;
    out.n_mats = (int)g.mats.size();
    out.mat_ids = g.mats;
    char key[40];
    snprintf(key, sizeof key, "%016llx", (unsigned long long)fnv1a(out.source));
    out.key = key;
    return out;
}

} // namespace pt
