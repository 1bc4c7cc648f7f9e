/*
 * pt_user_object.h -- the CSG node of a user-defined Object subclass
 * (pt_object_device; reference include/object.h:10-24: Object::
 * makeSpanIterator is virtual, so a caller may add shapes of its own).
 *
 * Appended to a scene's module by codegen.cpp only when the scene holds such
 * an object, after device/pt_device.h, whose node protocol it implements (see
 * Sph there): a leaf primitive with one span per ray.  The caller's bodies
 * arrive as B (codegen's UObjB_<id>):
 *     bool B::span(V3 o, V3 d, const float *prm, float &t0, float &t1)
 *         -- whether the ray o + t d (d not normalised) meets the object, and
 *            then its entry and exit parameters, t0 <= t1 (the reference
 *            Span's start and end, include/span.h:12-120);
 *     V3 B::normal(V3 p, const float *prm)
 *         -- the outward surface normal at p (the span's start normal at the
 *            entry point and end normal at the exit; traceRay flips the end
 *            normal, path-trace.h:89).
 * Every check the kernel's fast paths take is the conservative one for an
 * unknown shape: never dark (an emissive user object is always reachable),
 * "ends before EPS" only from the computed span itself.
 */
namespace ptd
{

template <int PRIM, int OFF, int MAT, class B>
struct UObj
{
    static constexpr int LO = PRIM, HI = PRIM + 1;
    static constexpr bool UNION_ONLY = true; /* a leaf: no Intersection / Difference at or below */
    static constexpr bool NO_DIFF = true;
    template <class PS>
    __device__ static __forceinline__ int isect_empty(const PS &) { return 1; }
    struct Ctx
    {
        V3 o; /* the query origin (in the object's frame) */
    };
    struct St
    {
        float t0, t1;
        int live;
    };
    __device__ static __forceinline__ void prep(Ctx &c, V3 o, const Env &) { c.o = univ(o); }
    __device__ static __forceinline__ void prep_l(Ctx &c, V3 o, const Env &) { c.o = o; }
    __device__ static __forceinline__ void init(St &s, const Ctx &c, const Ray &q, const Env &e)
    {
        float t0 = __builtin_nanf(""), t1 = __builtin_nanf("");
        const bool live = B::span(c.o, q.d, e.P + OFF, t0, t1);
        s.live = live ? 1 : 0;
        s.t0 = t0, s.t1 = t1;
    }
    __device__ static __forceinline__ bool pull(St &s, CS &out)
    {
        if (!s.live)
            return false;
        out.t0 = s.t0, out.t1 = s.t1;
        out.r0 = mkref(PRIM, MAT, 0), out.r1 = mkref(PRIM, MAT, 1);
        s.live = 0;
        return true;
    }
    template <class PS>
    __device__ static __forceinline__ void span(PS &ps, const Ctx &c, const Ray &q, const Env &e)
    {
        St s;
        init(s, c, q, e);
        ps.t0[PRIM] = s.t0, ps.t1[PRIM] = s.t1, ps.live[PRIM] = s.live;
    }
    template <class PS>
    __device__ static __forceinline__ void init_ps(St &s, const PS &ps)
    {
        s.t0 = ps.t0[PRIM], s.t1 = ps.t1[PRIM], s.live = ps.live[PRIM];
    }
    template <class F>
    __device__ static __forceinline__ void each_pos(F &&f) { f(IC<PRIM>(), IC<MAT>()); }
    template <class SEL, class PS>
    __device__ static __forceinline__ void span_sel(PS &ps, const Ctx &c, const Ray &q, const Env &e)
    {
        if constexpr (SEL::take(MAT))
            span(ps, c, q, e);
    }
    template <class SEL, class F>
    __device__ static __forceinline__ void each_sel(F &&f)
    {
        if constexpr (SEL::take(MAT))
            f(IC<PRIM>(), IC<MAT>());
    }
    /* lanes whose span is dead or ends before EPS, from the span itself */
    template <class SEL, bool NORM>
    __device__ static __forceinline__ u64 clear_mask(const Ctx &c, const Ray &q, const Env &e)
    {
        if constexpr (SEL::take(MAT))
            return ~0ull;
        St s;
        init(s, c, q, e);
        return __ballot(!s.live || s.t1 < EPS);
    }
    template <class SEL>
    __device__ static constexpr bool clear_ok() { return true; }
    template <class PS>
    __device__ static __forceinline__ int fast_ok(const PS &) { return 1; }
    __device__ static __forceinline__ V3 normal(int, float t, V3 o, V3 d, const Env &e)
    {
        return B::normal(o + t * d, e.P + OFF);
    }
    template <class SEL>
    __device__ static constexpr bool raw_ok() { return true; }
    template <class SEL>
    __device__ static constexpr int nsel() { return SEL::take(MAT) ? 1 : 0; }
    /* no direction is provably dark for an emissive shape the kernel cannot see into */
    template <class SEL>
    __device__ static __forceinline__ u64 dark_mask(const Ctx &, V3, const Env &)
    {
        if constexpr (!SEL::take(MAT))
            return ~0ull;
        return 0ull;
    }
    template <class SEL>
    __device__ static __forceinline__ bool dark_pre(const Ctx &, const Env &)
    {
        return true;
    }
};

} // namespace ptd
