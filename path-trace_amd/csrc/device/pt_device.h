/*
 * pt_device.h -- CDNA4 (gfx950) device library of the MI355X path tracer.
 *
 * Embedded verbatim into every scene module that the runtime generates and
 * compiles with hiprtc (runtime.cpp, codegen.cpp).  A scene module is this
 * header + one generated `struct Scene` whose geometry is a compile-time CSG
 * type (Sph/Pln/Uni/Isect/Diff/Xf nodes with their parameters at fixed offsets
 * of the scene parameter block P) and whose materials are compile-time texture
 * trees.  All per-scene control flow is therefore static and every node's
 * state lives in VGPRs; scene constants are scalar loads from P.
 *
 * Execution model (PT_WPW independent 64-lane waves per workgroup, each with
 * its own LDS work areas):
 *   - a wave dequeues a chunk of up to PT_CHUNK consecutive (pixel, sample)
 *     items; lane j traces item j's camera query and finishes the sample
 *     itself when its tree is that query plus at most one leaf mirror child
 *     (lane_sample); the other items are walked one after another by all 64
 *     lanes together with wave-uniform state (the "spine": camera ray, mirror
 *     and refraction chains, non-leaf children) and an explicit frame stack in
 *     LDS instead of the reference's recursion (include/path-trace.h:58-165);
 *   - a scatter loop with scatter_coefficient > eps (path-trace.h:138-163) is a
 *     BURST: each generation round evaluates 64*PT_KATT consecutive rejection
 *     attempts, PT_KATT per lane (attempt l + 64k, its stream position reached
 *     by O(1) LCG jumps), ballots accept / fail / non-leaf / dark masks,
 *     replays the reference's sequential consumption rule with scalar bit
 *     arithmetic, parks the accepted children that may be lit in an LDS ring
 *     and traces them 64 at a time, one child per lane, through a cascade of
 *     compacted passes (clear, fast, full merge);
 *   - a leaf child (depth-1 <= 0 or child strength < eps: path-trace.h:105-108)
 *     draws no random numbers, so children of a burst are independent and
 *     the RNG stream and every branch stay bit-identical to the reference.
 *
 * Arithmetic: compiled with -ffp-contract=off and correctly rounded f32
 * division/sqrt; every expression keeps the reference's evaluation order, so
 * per-sample radiance is bit-identical to the reference in PT_ORDER_REFERENCE
 * and to the oracle's fast order in the fast path (a burst's non-zero child
 * terms dealt round-robin to 64 lane sums, added as their 64-wide pairwise
 * tree).
 */
#ifndef PT_DEVICE_H
#define PT_DEVICE_H

typedef unsigned long long u64;
typedef unsigned int u32;

namespace ptd
{

constexpr float EPS = 1e-3f;      /* include/misc.h:7 */
constexpr float MAXV = 1e20f;     /* include/misc.h:8 */
constexpr u64 LCG_MULT = 214013ull; /* DefaultRandomEngine, include/path-trace.h:47 */
constexpr u64 LCG_INC = 2531011ull;  /* include/path-trace.h:47 */

/* -------------------------------------------------------------- launch --- */
struct PtImage
{
    const float4 *data; /* RGBA, row 0 = top */
    u32 w, h;
};

struct PtLaunch
{
    u64 seed;
    long long n_items;  /* items in this launch: slot-major, nsamp samples per slot */
    long long chunk0;   /* first chunk (64 items) of this launch                   */
    int W, H;
    float sw, sh, dist;
    int depth;
    int nsamp;          /* samples per pixel slot in this pass                     */
    int s0;             /* first sample index of this pass                         */
    int gw;             /* pixel index = py * gw + px (gw = W, or wider for the
                           adaptive caller's block-edge pixels)                   */
    int chunk;          /* items per work-queue dequeue, 1..64 (0 = PT_CHUNK)      */
    int sample_major;   /* item order: 1 = consecutive items are consecutive slots
                           at one sample, 0 = a slot's samples are consecutive    */
    int block_sums;     /* stage one partial per 32-sample block (slot-major,
                           chunk 32 or 64, nsamp % chunk == 0), else one value
                           per sample */
    long long perm;     /* sample-major: slot = (k * perm) mod nslots for the k-th
                           slot of a sample (perm coprime to nslots; 0 = k)      */
    const float *rays;  /* PT_RAYS modules (pt_trace_rays): slot k's ray, 7 floats
                           (origin, direction, strength) -- traceRay's arguments,
                           include/path-trace.h:59 -- instead of a camera ray    */
    long long ray0;     /* PT_RAYS: engine key index of slot 0 (slot k: ray0 + k) */
    int grab;           /* chunks a wave takes per work-queue atomic while plenty are
                           left (1 near the end of the launch); >= 1               */
    const unsigned *list; /* split launches (lane-walk scenes): the full kernel takes its
                           chunks from this list, stats[35] long (nullptr: every
                           chunk of the launch)                                   */
    unsigned *bail;     /* split launches: the light kernel appends the chunks it
                           leaves to the full kernel here (count: stats[35])      */
};
/* The engine key index of a slot's item: its pixel index, or in a ray-list
 * module the caller's ray index */
#ifdef PT_RAYS
#define PT_ITEM_KEY(lp, pix) ((u64)((lp).ray0 + (long long)(pix)))
#else
#define PT_ITEM_KEY(lp, pix) ((u64)(pix))
#endif

struct Env
{
    const float *__restrict__ P;
    const PtImage *__restrict__ img;
};

/* ---------------------------------------------------------------- math --- */
struct V3
{
    float x, y, z;
};
__device__ __forceinline__ V3 mk(float x, float y, float z)
{
    V3 r;
    r.x = x, r.y = y, r.z = z;
    return r;
}
__device__ __forceinline__ V3 operator+(V3 a, V3 b) { return mk(a.x + b.x, a.y + b.y, a.z + b.z); }
__device__ __forceinline__ V3 operator-(V3 a, V3 b) { return mk(a.x - b.x, a.y - b.y, a.z - b.z); }
__device__ __forceinline__ V3 operator*(V3 a, V3 b) { return mk(a.x * b.x, a.y * b.y, a.z * b.z); }
__device__ __forceinline__ V3 operator*(float s, V3 a) { return mk(a.x * s, a.y * s, a.z * s); }
__device__ __forceinline__ V3 operator/(V3 a, float s) { return mk(a.x / s, a.y / s, a.z / s); }
__device__ __forceinline__ V3 operator-(V3 a) { return mk(-a.x, -a.y, -a.z); }
__device__ __forceinline__ bool is_zero(V3 a) { return a.x == 0.0f && a.y == 0.0f && a.z == 0.0f; }
/* Vector3D dot: products then (x + y) + z, vector3d.h:102-106 */
__device__ __forceinline__ float dot(V3 a, V3 b) { return (a.x * b.x + a.y * b.y) + a.z * b.z; }
__device__ __forceinline__ float length(V3 v) { return __builtin_sqrtf(dot(v, v)); }
__device__ __forceinline__ V3 normalize(V3 v)
{
    float m = length(v);
    if (m == 0.0f)
        m = 1.0f;
    return v / m;
}
/* Exact fast paths for f32 sqrt and '/'.  LLVM lowers correctly rounded
 * sqrtf and '/' on gfx950 to fixed sequences (v_sqrt + ulp fix-up with
 * range scaling and a class check; v_div_scale / v_rcp / 5 FMAs /
 * v_div_fmas / v_div_fixup).  For operands in the ranges below the scaling
 * steps are the identity, so the remaining core -- copied instruction for
 * instruction -- returns the same bits; other operands take the full path.
 * pt_selftest_math() checks this on the GPU against the compiler's own
 * sqrtf and '/'. */
__device__ __forceinline__ float sqrt_core(float x)
{
    float s = __builtin_amdgcn_sqrtf(x);
    float sd = __uint_as_float(__float_as_uint(s) - 1u), su = __uint_as_float(__float_as_uint(s) + 1u);
    float rd = __builtin_fmaf(-sd, s, x), ru = __builtin_fmaf(-su, s, x);
    s = (rd <= 0.0f) ? sd : s;
    s = (ru > 0.0f) ? su : s;
    return s;
}
/* sqrt_core alone is exact for x >= 2^-96 (incl. +inf), x == +-0 and NaN. */
__device__ __forceinline__ bool sqrt_core_ok(float x) { return !(x < 0x1p-96f) || x == 0.0f; }
__device__ __forceinline__ float csqrt(float x) /* == __builtin_sqrtf(x), bitwise (checked by the self-test) */
{
    float s = sqrt_core(x);
    if (!sqrt_core_ok(x))
        s = __builtin_sqrtf(x);
    return s;
}
struct Rcp /* refined reciprocal of a denominator, shared by several quotients */
{
    float d, r;
};
__device__ __forceinline__ Rcp mkrcp(float d)
{
    Rcp R;
    R.d = d;
    float r = __builtin_amdgcn_rcpf(d);
    float e = __builtin_fmaf(-d, r, 1.0f);
    R.r = __builtin_fmaf(e, r, r);
    return R;
}
/* |x| in [2^-30, 2^30] for denominators, [2^-60, 2^60] for numerators: no
 * v_div_scale scaling (exponent gap < 96, no denormal operand/reciprocal/
 * quotient) and no v_div_fixup special case. */
__device__ __forceinline__ bool den_ok(float d)
{
    u32 b = __float_as_uint(d) & 0x7fffffffu;
    return b - 0x30800000u <= 0x4e800000u - 0x30800000u;
}
__device__ __forceinline__ bool num_ok(float n)
{
    u32 b = __float_as_uint(n) & 0x7fffffffu;
    return b - 0x21800000u <= 0x5d800000u - 0x21800000u;
}
__device__ __forceinline__ float div_core(float n, const Rcp &R)
{
    float q = n * R.r;
    float e = __builtin_fmaf(-R.d, q, n);
    q = __builtin_fmaf(e, R.r, q);
    e = __builtin_fmaf(-R.d, q, n);
    return __builtin_fmaf(e, R.r, q);
}
/* n / R.d, bitwise equal to the compiler's correctly rounded division;
 * `dok` = den_ok(R.d), evaluated once per denominator. */
__device__ __forceinline__ float cdiv(float n, const Rcp &R, bool dok)
{
    float q = div_core(n, R);
    if (!(dok && num_ok(n)))
        q = n / R.d;
    return q;
}
/* True on every lane when any active lane has p: a scalar (wave-uniform)
 * branch, so a rarely needed slow path costs one compare-and-branch instead
 * of exec-mask bookkeeping or an if-converted second evaluation. */
__device__ __forceinline__ bool wave_any(bool p) { return __ballot(p) != 0ull; }
/* Marks a rarely taken wave-uniform fallback block: the empty volatile asm
 * keeps LLVM from if-converting it, which would evaluate the slow exact
 * sequence (v_div_scale / v_div_fmas / v_div_fixup, scaled sqrt) on every
 * pass and select. */
#define PT_COLD() asm volatile("")


__device__ __forceinline__ V3 cnormalize(V3 v) /* == normalize(v), bitwise */
{
    const float x = dot(v, v);
    float m = sqrt_core(x);
    const bool sbad = !sqrt_core_ok(x);
    if (wave_any(sbad)) {
        PT_COLD();
        if (sbad)
            m = __builtin_sqrtf(x);
    }
    if (m == 0.0f)
        m = 1.0f;
    Rcp R = mkrcp(m);
    V3 q = mk(div_core(v.x, R), div_core(v.y, R), div_core(v.z, R));
    const bool dbad = !(den_ok(m) && num_ok(v.x) && num_ok(v.y) && num_ok(v.z));
    if (wave_any(dbad)) {
        PT_COLD();
        if (dbad)
            q = mk(v.x / m, v.y / m, v.z / m);
    }
    return q;
}
/* normalize() of a kept attempt's direction in a diffuse burst (scatter
 * coefficient 1: w = v, the unit-ball draw itself), where cnormalize's exact
 * fast sequence needs none of its fallbacks: the hemisphere test passed, so
 * n.w > EPS with |n| = 1 + O(2^-23) and |w|^2 >= 1e-6 > 2^-96 (sqrt_core_ok)
 * and 1e-3 < |w| < 1.01 (den_ok, and m != 0); each component is a u11 value,
 * +0 or of magnitude in [2^-24, 1] (num_ok, or a +0 numerator, whose quotient
 * div_core also gets exactly: +0).  Same bits as normalize(). */
#ifndef PT_KEPT_NORM
#define PT_KEPT_NORM 1
#endif
__device__ __forceinline__ V3 cnormalize_kept(V3 v)
{
#if PT_KEPT_NORM
    const Rcp R = mkrcp(sqrt_core(dot(v, v)));
    return mk(div_core(v.x, R), div_core(v.y, R), div_core(v.z, R));
#else
    return cnormalize(v);
#endif
}
/* normalize() where the device library needs it (normals, reflect / refract,
 * the spherical sky map): PT_FAST_NORM=1 takes the exact fast sequence (same
 * bits).  Off: same-box A/B (profiles/round5/ab_grab_fastnorm_c3_full.txt)
 * C5 -3.6 % (its lane walks carry the extra branches), C3 -0.8 %, C2 +1.2 %
 * -- the mirror-ball map's part, which PT_FAST_MIRRORBALL keeps */
#ifndef PT_FAST_NORM
#define PT_FAST_NORM 0
#endif
#ifndef PT_FAST_MIRRORBALL /* off: same-box C2 A/B -2.4 % .. +1.2 % (noise), profiles/round5/ab_grab_adaptive.txt */
#define PT_FAST_MIRRORBALL 0
#endif
#if PT_FAST_NORM
#define PT_NORM(v) cnormalize(v)
#else
#define PT_NORM(v) normalize(v)
#endif
/* (int)x as x86 cvttss2si: out-of-range and NaN give INT_MIN (the reference
 * runs on x86; v_cvt_i32_f32 would saturate / give 0). */
__device__ __forceinline__ int cvt_x86(float x)
{
    return (x != x || x >= 2147483648.0f || x < -2147483648.0f) ? (int)0x80000000 : (int)x;
}
__device__ __forceinline__ float clamp01(float x)
{
    float m = (x < 1.0f) ? x : 1.0f;  /* std::min(1.0f, x) */
    return (0.0f < m) ? m : 0.0f;     /* std::max(0.0f, m) */
}
/* Vector3D::reflect, vector3d.h:186-190 */
__device__ __forceinline__ V3 reflect(V3 d, V3 n)
{
    n = PT_NORM(n);
    return d - (2.0f * dot(d, n)) * n;
}
__device__ __forceinline__ bool bad_ior(float ior, V3 n, V3 d)
{
    return ior < EPS || ior > 1.0f / EPS || is_zero(n) || is_zero(d);
}
/* Vector3D::refractStrength, vector3d.h:191-202 -- the final sqrt(sqrt(x)) is
 * ::sqrt(double) in the reference build: two double roots, one rounding. */
__device__ __forceinline__ float refract_strength(V3 d, float ior, V3 n)
{
    if (bad_ior(ior, n, d))
        return 0.0f;
    n = PT_NORM(n);
    V3 inc = PT_NORM(d);
    float c = dot(inc, n);
    float r = 1.0f - ior * ior * (1.0f - c * c);
    if (r <= 0.0f)
        return 0.0f;
    return (float)__builtin_sqrt(__builtin_sqrt((double)r));
}
/* Vector3D::refract, vector3d.h:203-214 */
__device__ __forceinline__ V3 refract(V3 d, float ior, V3 n)
{
    if (bad_ior(ior, n, d))
        return mk(0, 0, 0);
    n = PT_NORM(n);
    V3 inc = PT_NORM(d);
    float c = dot(inc, n);
    float arg = 1.0f - ior * ior * (1.0f - c * c);
    if (arg < 0.0f)
        return mk(0, 0, 0);
#if PT_FAST_NORM
    return PT_NORM(ior * inc - (ior * c + csqrt(arg)) * n);
#else
    return PT_NORM(ior * inc - (ior * c + __builtin_sqrtf(arg)) * n);
#endif
}
/* Matrix::apply / applyNoTranslate, transform.h:408-421; m in ctor order */
__device__ __forceinline__ V3 m_apply(const float *__restrict__ m, V3 v)
{
    return mk(((v.x * m[0] + v.y * m[1]) + v.z * m[2]) + m[3], ((v.x * m[4] + v.y * m[5]) + v.z * m[6]) + m[7],
              ((v.x * m[8] + v.y * m[9]) + v.z * m[10]) + m[11]);
}
__device__ __forceinline__ V3 m_lin(const float *__restrict__ m, V3 v)
{
    return mk((v.x * m[0] + v.y * m[1]) + v.z * m[2], (v.x * m[4] + v.y * m[5]) + v.z * m[6],
              (v.x * m[8] + v.y * m[9]) + v.z * m[10]);
}

/* ----------------------------------------------------------------- rng --- */
/* The reference's DefaultRandomEngine recurrence with a per-(pixel, sample)
 * starting state -- include/pt/pt_engine.h is the specification. */
struct Rng
{
    u64 st; /* the increment is always LCG_INC (pt_engine.h) */
};
__device__ __forceinline__ u64 splitmix64(u64 x)
{
    u64 z = x + 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}
__device__ __forceinline__ u32 lcg_out(u64 updated) { return (u32)(updated >> 32); }
__device__ __forceinline__ void rng_seed(Rng &r, u64 seed, u64 pixel, u64 sample)
{
    u64 key = splitmix64(seed) ^ (pixel << 20) ^ sample;
    r.st = splitmix64(key);
}
__device__ __forceinline__ u32 rng_next(Rng &r)
{
    r.st = r.st * LCG_MULT + LCG_INC;
    return lcg_out(r.st);
}
/* One engine step on the state's 32-bit words: (lo * M + inc) gives the new
 * low word and a carry below 2^19; hi * M + carry gives the new high word
 * (the output).  Two 32x32->64 multiply-adds instead of a generic 64-bit
 * multiply; the same state mod 2^64. */
struct W2
{
    u32 lo, hi;
};
__device__ __forceinline__ W2 lcg_step(W2 s)
{
    const u64 t = (u64)s.lo * LCG_MULT + LCG_INC;
    const u32 hi = (u32)((u64)s.hi * LCG_MULT + (t >> 32));
    return {(u32)t, hi};
}
/* uniform_real_distribution<float>, vector3d.h:22-33, for (0,1) and (-1,1) */
__device__ __forceinline__ float u01(u32 o) { return (float)o / 4294967296.0f; }
/* uniform(-1, 1): (float)o / 2^32 * (1 - -1) + -1 (include/vector3d.h:14-34).
 * Both power-of-two scalings are exact for o >= 1 (and 0 stays 0), so one
 * multiply by 2^-31 gives the same bits. */
__device__ __forceinline__ float u11(u32 o) { return __builtin_fmaf((float)o, 0x1p-31f, -1.0f); } /* exact product: == mul then add */

/* --------------------------------------------------------- wave helpers --- */
__device__ __forceinline__ float rdlane(float v, int l)
{
    return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), l));
}
__device__ __forceinline__ int uni(int v) { return __builtin_amdgcn_readfirstlane(v); }
__device__ __forceinline__ float unif(float v) { return __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(v))); }
__device__ __forceinline__ V3 univ(V3 v) { return mk(unif(v.x), unif(v.y), unif(v.z)); }
/* all-ones if the wave-uniform p holds, else 0, by scalar arithmetic */
__device__ __forceinline__ u64 uni_mask(bool p) { return 0ull - (u64)(u32)uni(p ? 1 : 0); }
/* this lane's bit of the uniform mask m as 0 / 1: one v_cndmask on the mask */
__device__ __forceinline__ int lane_bit(u64 m)
{
    int r;
    asm("v_cndmask_b32_e64 %0, 0, 1, %1" : "=v"(r) : "s"(m));
    return r;
}
/* a where this lane's bit of the uniform mask m is set, else b: one v_cndmask on the mask */
__device__ __forceinline__ int mask_sel(u64 m, int a, int b)
{
    int r;
    asm("v_cndmask_b32_e64 %0, %2, %1, %3" : "=v"(r) : "v"(a), "v"(b), "s"(m));
    return r;
}
/* v + this lane's bit of the uniform mask m: one v_addc with m as carry-in */
__device__ __forceinline__ int add_lane_bit(int v, u64 m)
{
    int r;
    u64 co;
    asm("v_addc_co_u32_e64 %0, %1, %2, 0, %3" : "=v"(r), "=s"(co) : "v"(v), "s"(m));
    return r;
}
/* 0 where this lane's bit of the uniform mask m is set, else v */
__device__ __forceinline__ int zero_if(u64 m, int v)
{
    int r;
    asm("v_cndmask_b32_e64 %0, %1, 0, %2" : "=v"(r) : "v"(v), "s"(m));
    return r;
}
/* base + set bits of the uniform mask m in the lanes below this one (v_mbcnt) */
__device__ __forceinline__ int mbcnt(u64 m, int base)
{
    return (int)__builtin_amdgcn_mbcnt_hi((u32)(m >> 32), __builtin_amdgcn_mbcnt_lo((u32)m, (u32)base));
}
/* The lane index recomputed where it is used (v_mbcnt of all ones): an asm
 * the compiler can neither merge nor hoist, so no register holds it across a
 * burst -- where it was spilled to scratch in scenes under VGPR pressure. */
__device__ __forceinline__ int lane_id()
{
    int l;
    asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(l));
    return l;
}
/* this lane's bit of the uniform mask m, by arithmetic */
__device__ __forceinline__ bool lane_in(u64 m) { return (m >> (threadIdx.x & 63)) & 1ull; }
/* the same as a branch condition: `if (in_mask(m))` runs the block with exec = m
 * (s_and_saveexec on the mask itself, no per-lane compare).  The LLVM intrinsic
 * is named directly: the hiprtc front end lacks its clang builtin. */
extern "C" __device__ bool pt_llvm_inverse_ballot(u64) __asm("llvm.amdgcn.inverse.ballot.i64");
__device__ __forceinline__ bool in_mask(u64 m) { return pt_llvm_inverse_ballot(m); }
__device__ __forceinline__ int nth_set_bit(u64 m, int k) /* 1-based k, m has >= k bits */
{
    for (int j = 1; j < k; j++)
        m &= m - 1;
    return __builtin_ctzll(m);
}
/* 64-wide pairwise tree sum, identical in every lane: ((a0+a1)+(a2+a3))+...
 * Levels 1-4 run in DPP (quad_perm [1,0,3,2], [2,3,0,1], row_half_mirror,
 * row_mirror): after level k every aligned group of 2^k lanes holds the same
 * partial sum, so a mirror partner is as good as the xor partner and IEEE
 * commutativity makes each lane's sum bitwise equal.  The four row sums are
 * then combined as (r0 + r1) + (r2 + r3) through readlane -- no LDS traffic. */
template <int CTRL>
__device__ __forceinline__ float dpp_partner(float v)
{
    return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, 0xF, 0xF, false));
}
/* Inclusive prefix sum of v over the wave's lanes (lane l: v_0 + .. + v_l),
 * integer, so any association gives the same value: Hillis-Steele within each
 * row of 16 (row_shr 1, 2, 4, 8; lanes shifted in from outside the row read
 * 0), then row 0's total into rows 1 and 3 and row 1's running total into rows
 * 2 and 3 (row_bcast:15 / :31; the other rows add the old value 0).  Needs all
 * 64 lanes active. */
template <int CTRL, int ROWS>
__device__ __forceinline__ u32 dpp_u32(u32 v)
{
    return (u32)__builtin_amdgcn_update_dpp(0, (int)v, CTRL, ROWS, 0xF, true);
}
__device__ __forceinline__ u32 wave_incl_scan(u32 v)
{
    v += dpp_u32<0x111, 0xF>(v);
    v += dpp_u32<0x112, 0xF>(v);
    v += dpp_u32<0x114, 0xF>(v);
    v += dpp_u32<0x118, 0xF>(v);
    v += dpp_u32<0x142, 0xA>(v);
    v += dpp_u32<0x143, 0xC>(v);
    return v;
}
/* (v << 1) | this lane's bit of the uniform mask m: one v_addc (v + v + carry-in m).
 * Each active lane's result depends on its own v and bit `lane` of m only, not
 * on EXEC (the instruction writes nothing for inactive lanes, like any VALU
 * op), so the compiler may move or merge it as a pure value.  The call site
 * (the lane-major generation round) runs with all 64 lanes active. */
__device__ __forceinline__ u32 shl_lane_bit(u32 v, u64 m)
{
    u32 r;
    u64 co;
    asm("v_addc_co_u32_e64 %0, %1, %2, %2, %3" : "=v"(r), "=s"(co) : "v"(v), "s"(m));
    return r;
}
/* v + src broadcast from the last lane of the row(s) below, on rows ROWS only;
 * the other rows add -0.0f, which leaves every value (and the sign of 0) */
template <int CTRL, int ROWS>
__device__ __forceinline__ float dpp_bcast_add(float v)
{
    return v + __int_as_float(__builtin_amdgcn_update_dpp(__float_as_int(-0.0f), __float_as_int(v), CTRL, ROWS, 0xF,
                                                          false));
}
__device__ __forceinline__ float wave_tree_sum(float v)
{
    v = v + dpp_partner<0xB1>(v);  /* quad_perm [1,0,3,2]: lane ^ 1 */
    v = v + dpp_partner<0x4E>(v);  /* quad_perm [2,3,0,1]: lane ^ 2 */
    v = v + dpp_partner<0x141>(v); /* row_half_mirror: partner in the other quad of the 8 */
    v = v + dpp_partner<0x140>(v); /* row_mirror: partner in the other 8 of the row */
    /* rows now hold r0..r3 in every lane; row_bcast:15 gives rows 1 and 3
     * r1 + r0 and r3 + r2, row_bcast:31 gives row 3 (r3 + r2) + (r1 + r0):
     * by commutativity the bits of (r0 + r1) + (r2 + r3) */
    v = dpp_bcast_add<0x142, 0xA>(v);
    v = dpp_bcast_add<0x143, 0x8>(v);
    return rdlane(v, 63);
}

/* acc + wave_tree_sum(v), channel by channel (acc wave-uniform, added as
 * acc + sum: IEEE addition commutes), the three tree sums interleaved level by
 * level in one block so that each DPP read of a channel is two instructions
 * after that channel's previous write (the VALU -> DPP hazard) without nops.
 * The row-broadcast levels add in place under a row mask (rows 1 and 3, then
 * row 3): the masked rows keep their value, as the -0.0 padding of
 * dpp_bcast_add does.  Same tree, same bits as wave_tree_sum (checked by the
 * GPU parity tests against the oracle's fast order).  Needs all 64 lanes
 * active. */
__device__ __forceinline__ V3 wave_tree_sum3_add(V3 v, V3 acc)
{
    float x = v.x, y = v.y, z = v.z;
    u32 sx, sy, sz;
#define PT_DPP3(CTL) "v_add_f32_dpp %0, %0, %0 " CTL "\n\t"                       \
                     "v_add_f32_dpp %1, %1, %1 " CTL "\n\t"                       \
                     "v_add_f32_dpp %2, %2, %2 " CTL "\n\t"
    asm volatile("s_nop 1\n\t"
                 PT_DPP3("quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf")
                 PT_DPP3("quad_perm:[2,3,0,1] row_mask:0xf bank_mask:0xf")
                 PT_DPP3("row_half_mirror row_mask:0xf bank_mask:0xf")
                 PT_DPP3("row_mirror row_mask:0xf bank_mask:0xf")
                 PT_DPP3("row_bcast:15 row_mask:0xa bank_mask:0xf")
                 PT_DPP3("row_bcast:31 row_mask:0x8 bank_mask:0xf")
                 "v_add_f32 %0, %6, %0\n\t"
                 "v_add_f32 %1, %7, %1\n\t"
                 "v_add_f32 %2, %8, %2\n\t"
                 "s_nop 1\n\t"
                 "v_readlane_b32 %3, %0, 63\n\t"
                 "v_readlane_b32 %4, %1, 63\n\t"
                 "v_readlane_b32 %5, %2, 63"
                 : "+v"(x), "+v"(y), "+v"(z), "=s"(sx), "=s"(sy), "=s"(sz)
                 : "s"(acc.x), "s"(acc.y), "s"(acc.z));
#undef PT_DPP3
    return mk(__uint_as_float(sx), __uint_as_float(sy), __uint_as_float(sz));
}

/* ----------------------------------------------------------- CSG spans --- */
/* Compact span: a boundary is (t, ref); the reference's normal and material
 * (include/span.h:12-120) are functions of ref and recomputed only for the
 * chosen hit.  ref = prim << 14 | material << 2 | end << 1 | flip. */
struct CS
{
    float t0, t1;
    u32 r0, r1;
};
constexpr u32 FLIP = 1u;
__device__ __forceinline__ constexpr u32 mkref(int prim, int mat, int end)
{
    return ((u32)prim << 14) | ((u32)mat << 2) | ((u32)end << 1);
}
__device__ __forceinline__ int ref_mat(u32 r) { return (int)((r >> 2) & 0xFFFu); }
__device__ __forceinline__ int ref_prim(u32 r) { return (int)(r >> 14); }
__device__ __forceinline__ int ref_end(u32 r) { return (int)((r >> 1) & 1u); }
/* span.h:93-119; copyEndFromStart / copyStartFromEnd negate the normal */
__device__ __forceinline__ void end_from_end(CS &a, const CS &b) { a.t1 = b.t1, a.r1 = b.r1; }
__device__ __forceinline__ void end_from_start(CS &a, const CS &b) { a.t1 = b.t0, a.r1 = b.r0 ^ FLIP; }
__device__ __forceinline__ void start_from_end(CS &a, const CS &b) { a.t0 = b.t1, a.r0 = b.r1 ^ FLIP; }
__device__ __forceinline__ void start_from_start(CS &a, const CS &b) { a.t0 = b.t0, a.r0 = b.r0; }

/* One query direction as every primitive of a traversal sees it: |d|^2 and
 * its refined reciprocal are shared (the sphere quotients all divide by a). */
#ifdef PT_NO_AXIS_SHARE /* A/B hook: every plane takes its own reciprocal */
#undef PT_AXIS_SHARE
#endif
struct Ray
{
    V3 d;
    float a;
    Rcp ra;
    int aok; /* den_ok(a) */
#ifdef PT_AXIS_SHARE
    /* direction components k of PT_AXIS_SHARE: their refined reciprocals and
     * den_ok, shared by the unit-normal planes of axis k (Pln UNIT) */
    Rcp rk[3];
    int rkok[3];
#endif
};
__device__ __forceinline__ Ray mkray(V3 d)
{
    Ray q;
    q.d = d;
    q.a = dot(d, d);
    q.ra = mkrcp(q.a);
    q.aok = den_ok(q.a) ? 1 : 0;
#ifdef PT_AXIS_SHARE
    const float dk[3] = {d.x, d.y, d.z};
#pragma unroll
    for (int k = 0; k < 3; k++)
        if ((PT_AXIS_SHARE >> k) & 1) {
            q.rk[k] = mkrcp(dk[k]);
            q.rkok[k] = den_ok(dk[k]) ? 1 : 0;
        }
#endif
    return q;
}
/* The same for a normalised direction (the burst passes' children): |d|^2 is
 * 1 within 1e-6, so den_ok(a) holds and the spans' quotient checks fold */
#ifndef PT_UNIT_RAY
#define PT_UNIT_RAY 1
#endif
__device__ __forceinline__ Ray mkray_unit(V3 d)
{
    Ray q = mkray(d);
#if PT_UNIT_RAY
    q.aok = 1;
#endif
    return q;
}

/* ---- fast first-hit ----------------------------------
 * Every primitive contributes at most one span.  When every pair of spans that
 * meets at a merge node (x from the node's A side, y from its B side, each a
 * "positive" primitive of that side: one reachable through Union children,
 * Difference A sides and TransformedObjects, not through an Intersection) is
 * either strictly separated or lies entirely before EPS, the lazy merges pass
 * every positive span through unchanged apart from spans ending before EPS,
 * which traceRay's scan skips.  The first qualifying span of the root is then
 * the live positive span with t1 >= EPS and the smallest t0, and the scan's
 * tests (path-trace.h:66-100) apply to it alone.  Lanes that fail the check
 * take the full merge; both give the same bits. */
template <int V>
struct IC
{
    static constexpr int value = V;
};
template <int NP>
struct PrimSpans
{
    float t0[NP], t1[NP];
    int live[NP];
};
template <class PS>
__device__ __forceinline__ int sep(const PS &ps, int x, int y)
{
    return (!ps.live[x]) | (!ps.live[y]) | (ps.t1[x] < ps.t0[y]) | (ps.t1[y] < ps.t0[x]) |
           ((ps.t1[x] < EPS) & (ps.t1[y] < EPS));
}
/* At a Union node (src/union.cpp:84-134) overlapping spans merge into one
 * whose start is the earlier start (the B side's on a tie, :125-132); when
 * both starts are >= EPS and differ, that merged span begins at the smaller
 * start >= EPS, so traceRay's scan stops at it exactly as at the earlier
 * span alone -- what fast_first_hit picks.  (A third span separated from both
 * lies wholly before or after their merge.)  Such pairs pass too: unions of
 * overlapping half-spaces (C2/C5's sky box, ground planes) stay on the fast
 * pass.
 * At a Difference node (src/difference.cpp:84-135) a B span y that starts
 * strictly after an A span x starting at >= EPS cuts x to [x0, y0] (and
 * maybe [y1, x1] after it): the output still begins at x's own start, and
 * the part before it is a subset of x, so every check made against x above
 * stays valid.  (y starting at or before x0 -- B covering x, or the :124-130
 * quirk's inverted span -- keeps the strict rule.)  Intersection nodes keep
 * the strict rule: separation there means an empty intersection. */
/* A positive span that ends before EPS (a ray leaving the surface it starts
 * on) is inert: every span the merges above derive from it ends before EPS
 * too -- a Union merge with a span y that reaches EPS ends at y's end with
 * y's ref and starts before EPS like y (src/union.cpp:105-132), a Difference
 * only cuts it (its pieces, and the :124-130 quirk's inverted span, end at or
 * before its end), and the B spans a Difference consumes while passing it end
 * before it, i.e. before any later A span that the checks keep apart from it.
 * The scan (path-trace.h:66-100) skips spans ending before EPS, so the pair
 * checks may ignore it (the first-hit choice never takes it: its t1 < EPS).
 * Only positives: a B-side span that ends before EPS can still trigger the
 * quirk on the A span it overlaps. */
enum { NODE_ISECT = 0, NODE_UNION = 1, NODE_DIFF = 2 };
#ifndef PT_INERT
#define PT_INERT 1
#endif
template <class PS>
__device__ __forceinline__ int inert(const PS &ps, int x)
{
    return PT_INERT ? ps.live[x] & (ps.t1[x] < EPS) : 0;
}
template <int KIND, class PS>
__device__ __forceinline__ int pair_ok(const PS &ps, int x, int y)
{
    int ok = sep(ps, x, y);
    if (KIND == NODE_UNION)
        ok |= ((ps.t0[x] >= EPS) & (ps.t0[y] >= EPS) & (ps.t0[x] != ps.t0[y])) | inert(ps, x) | inert(ps, y);
    if (KIND == NODE_DIFF)
        ok |= ((ps.t0[x] >= EPS) & (ps.t0[y] > ps.t0[x])) | inert(ps, x);
    return ok;
}

/* Selects every primitive (each_sel) */
struct AllPrims
{
    __device__ static constexpr bool take(int) { return true; }
};

/* Sphere (src/sphere.cpp:31-49).  P[OFF..OFF+3] = center, r*r.  Branch-free:
 * t0/t1 are computed on every lane (dead lanes' values are never read), with
 * one wave-uniform fallback for operands outside the exact fast paths. */
#ifndef PT_SPHERE_SKIP
#define PT_SPHERE_SKIP 0
#endif
template <int PRIM, int OFF, int MAT>
struct Sph
{
    static constexpr int LO = PRIM, HI = PRIM + 1;
    static constexpr bool UNION_ONLY = true; /* no Intersection / Difference at or below */
    static constexpr bool NO_DIFF = true; /* no Difference at or below */
    template <class PS>
    __device__ static __forceinline__ int isect_empty(const PS &) { return 1; }
    struct Ctx
    {
        V3 omc;
        float c;
        float thr; /* clear_mask's bound on b for a normalised direction */
    };
    struct St
    {
        float t0, t1;
        int live; /* int, not bool: kept in a VGPR instead of an SGPR lane mask */
    };
    /* clear_mask: for a direction d with |d|^2 = a in 1 +- 2^-20 the span ends
     * before EPS whenever b = (o - c).d >= thr:
     *  - c > 0 (origin outside), thr = 0: fl(a*c) >= 0 makes disc <= fl(b*b),
     *    so sqrt(disc) <= sqrt(fl(b*b)) = b and t1 = (-b + sqrt(disc)) / a <= 0;
     *  - c <= 0 (origin on or inside: the burst origin's own sphere), thr =
     *    527 |c| and b <= r <= 99: -b + sqrt(disc) is exact (Sterbenz) and at
     *    most (2u + u^2) b + (1 + u)^2 a |c| / (2b), so t1 <= 2u b / a +
     *    (1 + 3u) |c| / (2b) < 1.2e-5 + 9.5e-4 < EPS (u = 2^-24).
     * NaN c gives a NaN threshold: never clear. */
    __device__ static __forceinline__ float clear_thr(float c, const Env &e)
    {
        return c > 0.0f ? 0.0f : e.P[OFF + 3] < 9801.0f ? -c * 527.0f : __builtin_inff();
    }
    __device__ static __forceinline__ void prep(Ctx &c, V3 o, const Env &e)
    {
        c.omc = univ(o - mk(e.P[OFF], e.P[OFF + 1], e.P[OFF + 2]));
        c.c = unif(dot(c.omc, c.omc) - e.P[OFF + 3]);
        c.thr = unif(clear_thr(c.c, e));
    }
    /* the same for a per-lane origin */
    __device__ static __forceinline__ void prep_l(Ctx &c, V3 o, const Env &e)
    {
        c.omc = o - mk(e.P[OFF], e.P[OFF + 1], e.P[OFF + 2]);
        c.c = dot(c.omc, c.omc) - e.P[OFF + 3];
        c.thr = clear_thr(c.c, e);
    }
    __device__ static __forceinline__ void init(St &s, const Ctx &c, const Ray &q, const Env &)
    {
        const float b = dot(c.omc, q.d);
        const float disc = b * b - q.a * c.c;
#if PT_RECEDE_DEAD
        /* Experiment hook, off: exact, but C2 -4 % (the waves whose only live
         * lanes recede are rare; profiles/round6/ab_recede_dead_c2_not_kept.txt).
         * Union-only trees: a sphere the ray leaves from outside
         * (c > 0, b >= 0) has t1 <= 0 -- fl(a*c) >= 0 makes disc <= fl(b*b),
         * so sqrt(disc) <= b -- and a span ending before EPS changes no union
         * result: the union rule never takes it, and in the lazy merge it can
         * only join spans that start before EPS, whose ends (and end normals)
         * it never supplies (src/union.cpp:84-134, path-trace.h:66-100).  Such
         * a lane counts as dead, so a wave whose other lanes miss skips the
         * root and the divisions. */
        const bool live = !(disc <= EPS) && !(c.c > 0.0f && b >= 0.0f);
#else
        const bool live = !(disc <= EPS);
#endif
#if PT_SPHERE_SKIP
        /* no lane meets the sphere: skip the root and the divisions (a dead
         * span's bounds are never read) */
        if (!wave_any(live)) {
            s.live = 0;
            s.t0 = s.t1 = __builtin_nanf("");
            return;
        }
#endif
        const float sq = sqrt_core(disc); /* exact: disc > EPS (or inf/NaN) where live */
        const float n0 = -b - sq, n1 = -b + sq;
        float t0 = div_core(n0, q.ra), t1 = div_core(n1, q.ra);
        const bool bad = live && !(q.aok && num_ok(n0) && num_ok(n1));
        if (wave_any(bad)) {
        PT_COLD();
            if (bad)
                t0 = n0 / q.a, t1 = n1 / q.a;
        }
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
    /* init() from the span span() already computed (the same values) */
    template <class PS>
    __device__ static __forceinline__ void init_ps(St &s, const PS &ps)
    {
        s.t0 = ps.t0[PRIM], s.t1 = ps.t1[PRIM], s.live = ps.live[PRIM];
    }
    template <class F>
    __device__ static __forceinline__ void each_pos(F &&f) { f(IC<PRIM>(), IC<MAT>()); }
    /* the same for primitives whose material SEL selects, all primitives not just positive ones */
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
    /* Lanes whose span is dead or provably ends before EPS (unselected
     * primitives only; NORM: q.d is a normalised direction, see clear_thr) */
    template <class SEL, bool NORM>
    __device__ static __forceinline__ u64 clear_mask(const Ctx &c, const Ray &q, const Env &)
    {
        if constexpr (SEL::take(MAT))
            return ~0ull;
        const float b = dot(c.omc, q.d);
        const float disc = b * b - q.a * c.c;
        const float thr = NORM ? c.thr : (c.c > 0.0f ? 0.0f : __builtin_inff());
        return __ballot(disc <= EPS) | __ballot(b >= thr);
    }
    template <class SEL>
    __device__ static constexpr bool clear_ok() { return true; }
    template <class PS>
    __device__ static __forceinline__ int fast_ok(const PS &) { return 1; }
    __device__ static __forceinline__ V3 normal(int, float t, V3 o, V3 d, const Env &e)
    {
        return PT_NORM((o + t * d) - mk(e.P[OFF], e.P[OFF + 1], e.P[OFF + 2]));
    }
    /* Sound test on an UNNORMALISED direction w that the span of normalize(w)
     * is dead or ends before EPS (the generation round's dark test).  Origin
     * outside (c > 0) and receding (b > 0): disc = fl(fl(b*b) - a*c) <= fl(b*b),
     * so sqrt(disc) <= b and t1 = (-b + sqrt(disc)) / a <= 0.  b's sign is
     * read off B = omc.w with a margin (1e-6 of sum |omc_i w_i|) that covers
     * the rounding of normalize() and of both dot products. */
    template <class SEL>
    __device__ static constexpr bool raw_ok() { return true; }
    template <class SEL>
    __device__ static constexpr int nsel() { return SEL::take(MAT) ? 1 : 0; }
    /* The test as a wave mask, one ballot per compare (a ballot of a combined
     * predicate is lowered through a v_cndmask / v_cmp round trip) */
    template <class SEL>
    __device__ static __forceinline__ u64 dark_mask(const Ctx &c, V3 w, const Env &)
    {
        if constexpr (!SEL::take(MAT))
            return ~0ull;
        const float B = dot(c.omc, w);
        const float s = (__builtin_fabsf(c.omc.x * w.x) + __builtin_fabsf(c.omc.y * w.y)) +
                        __builtin_fabsf(c.omc.z * w.z);
        return __ballot(B > __builtin_fmaxf(1e-6f * s, 1e-30f));
    }
    /* The test's burst-uniform precondition, taken once per burst (the dark
     * mask of a direction is dark_mask(w) & dark_pre: a scalar mask, neither a
     * ballot of pre && x -- InstCombine folds ballot(a) & ballot(b) into that
     * -- nor a branch, which would split the round's interleaved attempts) */
    template <class SEL>
    __device__ static __forceinline__ bool dark_pre(const Ctx &c, const Env &)
    {
        if constexpr (!SEL::take(MAT))
            return true;
        return c.c > 0.0f && (__builtin_fabsf(c.omc.x) + __builtin_fabsf(c.omc.y)) + __builtin_fabsf(c.omc.z) < 1e15f;
    }
};

/* Plane half-space {p : n.p + d < 0} (src/plane.cpp:35-63).  P[OFF..] = n, d. */
#ifndef PT_PLANE_AXIS_DARK
#define PT_PLANE_AXIS_DARK 1
#endif
#ifndef PT_PLANE_AXIS_DIV
#define PT_PLANE_AXIS_DIV 1 /* an axis-aligned plane's d.n as one product */
#endif
/* AX >= 0: the normal has one nonzero component, axis AX >> 1, negative if
 * AX & 1 (codegen knows the scene's numbers); -1 otherwise. */
/* UNIT: the normal is +-e_(AX >> 1) exactly and the scene has another such
 * plane on that axis (codegen PT_AXIS_SHARE): div = +-d_k, and the quotient
 * num / div is +-(num / d_k) -- IEEE division is sign-symmetric -- taken
 * with the ray's shared reciprocal of d_k. */
template <int PRIM, int OFF, int MAT, int AX = -1, int UNIT = 0>
struct Pln
{
    static constexpr int LO = PRIM, HI = PRIM + 1;
    static constexpr bool UNION_ONLY = true; /* no Intersection / Difference at or below */
    static constexpr bool NO_DIFF = true; /* no Difference at or below */
    template <class PS>
    __device__ static __forceinline__ int isect_empty(const PS &) { return 1; }
    struct Ctx
    {
        float num;
    };
    struct St
    {
        float t0, t1;
        int live; /* int, not bool: kept in a VGPR instead of an SGPR lane mask */
    };
    __device__ static __forceinline__ void prep(Ctx &c, V3 o, const Env &e)
    {
        c.num = unif(-e.P[OFF + 3] - dot(o, mk(e.P[OFF], e.P[OFF + 1], e.P[OFF + 2])));
    }
    __device__ static __forceinline__ void prep_l(Ctx &c, V3 o, const Env &e)
    {
        c.num = -e.P[OFF + 3] - dot(o, mk(e.P[OFF], e.P[OFF + 1], e.P[OFF + 2]));
    }
    __device__ static __forceinline__ void init(St &s, const Ctx &c, const Ray &q, const Env &e)
    {
        float div;
        if constexpr (AX >= 0 && PT_PLANE_AXIS_DIV) {
            /* one nonzero component: (d.x n.x + d.y n.y) + d.z n.z is that
             * component's product plus signed zeros -- the product itself
             * whenever it is nonzero, and a zero either way when it is zero
             * (which makes the plane degenerate, |div| < eps^2, regardless of
             * its sign).  Directions are finite (camera rays, normalised
             * children, reflections of them). */
            const float dc = (AX >> 1) == 0 ? q.d.x : (AX >> 1) == 1 ? q.d.y : q.d.z;
            div = dc * e.P[OFF + (AX >> 1)];
        } else {
            div = dot(q.d, mk(e.P[OFF], e.P[OFF + 1], e.P[OFF + 2]));
        }
        const bool small = __builtin_fabsf(div) < EPS * EPS;
        float t;
        bool bad;
#ifdef PT_AXIS_SHARE
        if constexpr (UNIT != 0 && AX >= 0) {
            /* e.P[OFF + k] is +-1: div == +-d_k exactly, |div| == |d_k| */
            const float q0 = div_core(c.num, q.rk[AX >> 1]);
            t = (AX & 1) ? -q0 : q0;
            bad = !small && !(q.rkok[AX >> 1] && num_ok(c.num));
        } else
#endif
        {
            t = div_core(c.num, mkrcp(div));
            bad = !small && !(den_ok(div) && num_ok(c.num));
        }
        if (wave_any(bad)) {
        PT_COLD();
            if (bad)
                t = c.num / div;
        }
        const bool deg = small || __builtin_fabsf(t) >= MAXV;
        const bool neg = div < 0.0f;
        s.live = (!deg || __builtin_fabsf(c.num) < EPS * EPS) ? 1 : 0;
        s.t0 = (!deg && neg) ? t : -MAXV;
        s.t1 = (!deg && !neg) ? t : MAXV;
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
    /* init() from the span span() already computed (the same values) */
    template <class PS>
    __device__ static __forceinline__ void init_ps(St &s, const PS &ps)
    {
        s.t0 = ps.t0[PRIM], s.t1 = ps.t1[PRIM], s.live = ps.live[PRIM];
    }
    template <class F>
    __device__ static __forceinline__ void each_pos(F &&f) { f(IC<PRIM>(), IC<MAT>()); }
    /* the same for primitives whose material SEL selects, all primitives not just positive ones */
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
    template <class SEL, bool NORM>
    __device__ static __forceinline__ u64 clear_mask(const Ctx &c, const Ray &q, const Env &e)
    {
        if constexpr (SEL::take(MAT))
            return ~0ull;
        St s;
        init(s, c, q, e);
        return __ballot(!s.live) | __ballot(s.t1 < EPS);
    }
    template <class SEL>
    __device__ static constexpr bool clear_ok() { return true; }
    template <class PS>
    __device__ static __forceinline__ int fast_ok(const PS &) { return 1; }
    __device__ static __forceinline__ V3 normal(int, float, V3, V3, const Env &e)
    {
        return PT_NORM(mk(e.P[OFF], e.P[OFF + 1], e.P[OFF + 2]));
    }
    /* Sound dark test on an unnormalised direction w (see Sph::dark_mask).
     * With num <= -1e-6 the span of normalize(w) is dead or ends before EPS
     * unless div = n.normalize(w) <= -1e-6: div in (-1e-6, 1e-6) is
     * degenerate (dead), div >= 1e-6 gives t1 = num / div < 0 (or |t| >= 1e20,
     * dead).  For |n|_1 <= 1.5 the computed div lies within 6.1e-7 |n|_1 <
     * 1e-6 of (n.w) / |w| for a computed n.w >= 0, so n.w >= 0 suffices. */
    template <class SEL>
    __device__ static constexpr bool raw_ok() { return true; }
    template <class SEL>
    __device__ static constexpr int nsel() { return SEL::take(MAT) ? 1 : 0; }
    template <class SEL>
    __device__ static __forceinline__ bool dark_pre(const Ctx &c, const Env &e)
    {
        if constexpr (!SEL::take(MAT))
            return true;
        const V3 np = mk(e.P[OFF], e.P[OFF + 1], e.P[OFF + 2]);
        return c.num <= -(EPS * EPS) && (__builtin_fabsf(np.x) + __builtin_fabsf(np.y)) + __builtin_fabsf(np.z) <= 1.5f;
    }
    template <class SEL>
    __device__ static __forceinline__ u64 dark_mask(const Ctx &, V3 w, const Env &e)
    {
        if constexpr (!SEL::take(MAT))
            return ~0ull;
        const V3 np = mk(e.P[OFF], e.P[OFF + 1], e.P[OFF + 2]);
        if constexpr (AX >= 0 && PT_PLANE_AXIS_DARK) {
            /* the exact n.w is n_a * w_a: its sign test is one compare (the
             * bound above holds for an exact n.w >= 0 as for a computed one) */
            const float wa = (AX >> 1) == 0 ? w.x : (AX >> 1) == 1 ? w.y : w.z;
            return __ballot((AX & 1) ? wa <= 0.0f : wa >= 0.0f);
        }
        return __ballot(dot(w, np) >= 0.0f);
    }
};

/* Binary CSG nodes: pull-protocol restatement of the reference iterators.
 * init() preloads the first span of each child (the reference's nextA(),
 * nextB() in init); pull() is the body of next() producing one span. */
#define PTD_BINARY_COMMON                                                                           \
    static constexpr int LO = A::LO, HI = B::HI;                                                    \
    struct Ctx                                                                                      \
    {                                                                                               \
        typename A::Ctx a;                                                                          \
        typename B::Ctx b;                                                                          \
    };                                                                                              \
    struct St                                                                                       \
    {                                                                                               \
        typename A::St a;                                                                           \
        typename B::St b;                                                                           \
        CS sa, sb;                                                                                  \
        int ea, eb; /* ints: VGPRs rather than SGPR lane masks */                                  \
    };                                                                                              \
    __device__ static __forceinline__ void prep(Ctx &c, V3 o, const Env &e)                        \
    {                                                                                               \
        A::prep(c.a, o, e);                                                                         \
        B::prep(c.b, o, e);                                                                         \
    }                                                                                               \
    __device__ static __forceinline__ void prep_l(Ctx &c, V3 o, const Env &e)                      \
    {                                                                                               \
        A::prep_l(c.a, o, e);                                                                       \
        B::prep_l(c.b, o, e);                                                                       \
    }                                                                                               \
    __device__ static __forceinline__ void init(St &s, const Ctx &c, const Ray &q, const Env &e)   \
    {                                                                                               \
        A::init(s.a, c.a, q, e);                                                                    \
        B::init(s.b, c.b, q, e);                                                                    \
        s.ea = !A::pull(s.a, s.sa);                                                                 \
        s.eb = !B::pull(s.b, s.sb);                                                                 \
    }                                                                                               \
    template <class PS>                                                                             \
    __device__ static __forceinline__ void span(PS &ps, const Ctx &c, const Ray &q, const Env &e)  \
    {                                                                                               \
        A::span(ps, c.a, q, e);                                                                     \
        B::span(ps, c.b, q, e);                                                                     \
    }                                                                                               \
    template <class PS>                                                                             \
    __device__ static __forceinline__ void init_ps(St &s, const PS &ps)                            \
    {                                                                                               \
        A::init_ps(s.a, ps);                                                                        \
        B::init_ps(s.b, ps);                                                                        \
        s.ea = !A::pull(s.a, s.sa);                                                                 \
        s.eb = !B::pull(s.b, s.sb);                                                                 \
    }                                                                                               \
    template <class SEL, class PS>                                                                  \
    __device__ static __forceinline__ void span_sel(PS &ps, const Ctx &c, const Ray &q, const Env &e) \
    {                                                                                               \
        A::template span_sel<SEL>(ps, c.a, q, e);                                                   \
        B::template span_sel<SEL>(ps, c.b, q, e);                                                   \
    }                                                                                               \
    template <class SEL, class F>                                                                   \
    __device__ static __forceinline__ void each_sel(F &&f)                                          \
    {                                                                                               \
        A::template each_sel<SEL>(f);                                                               \
        B::template each_sel<SEL>(f);                                                               \
    }                                                                                               \
    template <class SEL, bool NORM>                                                                 \
    __device__ static __forceinline__ u64 clear_mask(const Ctx &c, const Ray &q, const Env &e)     \
    {                                                                                               \
        return A::template clear_mask<SEL, NORM>(c.a, q, e) & B::template clear_mask<SEL, NORM>(c.b, q, e); \
    }                                                                                               \
    template <class PS>                                                                             \
    __device__ static __forceinline__ int fast_ok(const PS &ps)                                     \
    {                                                                                               \
        int ok = A::fast_ok(ps) & B::fast_ok(ps);                                                   \
        A::each_pos([&](auto x, auto) { B::each_pos([&](auto y, auto) { ok &= pair_ok<KIND>(ps, decltype(x)::value, decltype(y)::value); }); }); \
        return ok;                                                                                  \
    }                                                                                               \
    __device__ static __forceinline__ V3 normal(int prim, float t, V3 o, V3 d, const Env &e)       \
    {                                                                                               \
        if (prim < A::HI)                                                                           \
            return A::normal(prim, t, o, d, e);                                                     \
        return B::normal(prim, t, o, d, e);                                                         \
    }                                                                                               \
    template <class SEL>                                                                            \
    __device__ static constexpr bool raw_ok() { return A::template raw_ok<SEL>() && B::template raw_ok<SEL>(); } \
    template <class SEL>                                                                            \
    __device__ static constexpr int nsel() { return A::template nsel<SEL>() + B::template nsel<SEL>(); } \
    template <class SEL>                                                                            \
    __device__ static __forceinline__ u64 dark_mask(const Ctx &c, V3 w, const Env &e)              \
    {                                                                                               \
        return A::template dark_mask<SEL>(c.a, w, e) & B::template dark_mask<SEL>(c.b, w, e);       \
    }                                                                                               \
    template <class SEL>                                                                            \
    __device__ static __forceinline__ bool dark_pre(const Ctx &c, const Env &e)                    \
    {                                                                                               \
        return A::template dark_pre<SEL>(c.a, e) && B::template dark_pre<SEL>(c.b, e);              \
    }

/* Each merge step decides what to emit and which child to advance, then
 * advances each child at exactly ONE call site: the inlined code of a CSG
 * tree stays linear in its node count instead of multiplying per level.
 * PT_PULL_SELECT: the step's span copies as value selects.  The branchy form
 * copies spans through a pointer the branch picks (out = s.sa / s.sb), which
 * keeps the whole iterator state in private memory (scratch); the select form
 * keeps it in registers.  That pays where the lazy merge is on the hot path
 * (lane walks: C5's private segment 776 -> 100 B) and costs registers where it
 * is rare (burst slow passes). */
#ifndef PT_PULL_SELECT
#if defined(PT_LANE_WALK)
#define PT_PULL_SELECT 1
#else
#define PT_PULL_SELECT 0
#endif
#endif

/* src/union.cpp:84-134 */
template <class A, class B>
struct Uni
{
    static constexpr int KIND = NODE_UNION;
    static constexpr bool UNION_ONLY = A::UNION_ONLY && B::UNION_ONLY;
    static constexpr bool NO_DIFF = A::NO_DIFF && B::NO_DIFF;
    template <class PS>
    __device__ static __forceinline__ int isect_empty(const PS &ps) { return A::isect_empty(ps) & B::isect_empty(ps); }
    PTD_BINARY_COMMON
    template <class SEL>
    __device__ static constexpr bool clear_ok() { return A::template clear_ok<SEL>() && B::template clear_ok<SEL>(); }
    template <class F>
    __device__ static __forceinline__ void each_pos(F &&f)
    {
        A::each_pos(f);
        B::each_pos(f);
    }
#if PT_PULL_SELECT
    __device__ static __forceinline__ bool pull(St &s, CS &out)
    {
        for (;;) {
            if (s.ea && s.eb)
                return false;
            /* the step's decisions as values: the span copies are selects,
             * never a copy through a pointer chosen by the branch (which
             * keeps the iterator state out of registers) */
            const bool ea = s.ea, eb = s.eb, both = !ea && !eb;
            const float a0 = s.sa.t0, a1 = s.sa.t1, b0 = s.sb.t0, b1 = s.sb.t1;
            const u32 ra0 = s.sa.r0, ra1 = s.sa.r1, rb0 = s.sb.r0, rb1 = s.sb.r1;
            const bool sepA = both && a1 < b0, sepB = both && !(a1 < b0) && b1 < a0;
            const bool over = both && !(a1 < b0) && !(b1 < a0);
            const bool aFirst = over && a0 < b0, bFirst = over && !(a0 < b0);
            const bool takeA = (!ea && eb) || sepA;
            const bool emit = ea || takeA || sepB;
            const bool adv_a = takeA || bFirst;
            out.t0 = takeA ? a0 : b0, out.t1 = takeA ? a1 : b1;
            out.r0 = takeA ? ra0 : rb0, out.r1 = takeA ? ra1 : rb1;
            const bool extA = aFirst && a1 < b1, extB = bFirst && a1 > b1; /* end_from_end */
            s.sa.t1 = extA ? b1 : a1, s.sa.r1 = extA ? rb1 : ra1;
            s.sb.t1 = extB ? a1 : b1, s.sb.r1 = extB ? ra1 : rb1;
            if (adv_a)
                s.ea = !A::pull(s.a, s.sa);
            else
                s.eb = !B::pull(s.b, s.sb);
            if (emit)
                return true;
        }
    }
#else
    __device__ static __forceinline__ bool pull(St &s, CS &out)
    {
        for (;;) {
            if (s.ea && s.eb)
                return false;
            bool emit = true, adv_a = false;
            if (s.ea) {
                out = s.sb;
            } else if (s.eb) {
                out = s.sa, adv_a = true;
            } else if (s.sa.t1 < s.sb.t0) {
                out = s.sa, adv_a = true;
            } else if (s.sb.t1 < s.sa.t0) {
                out = s.sb;
            } else if (s.sa.t0 < s.sb.t0) {
                if (s.sa.t1 < s.sb.t1)
                    end_from_end(s.sa, s.sb);
                emit = false;
            } else {
                if (s.sa.t1 > s.sb.t1)
                    end_from_end(s.sb, s.sa);
                emit = false, adv_a = true;
            }
            if (adv_a)
                s.ea = !A::pull(s.a, s.sa);
            else
                s.eb = !B::pull(s.b, s.sb);
            if (emit)
                return true;
        }
    }
#endif
};

/* src/intersection.cpp:84-130 */
template <class A, class B>
struct Isect
{
    static constexpr int KIND = NODE_ISECT;
    static constexpr bool UNION_ONLY = false;
    static constexpr bool NO_DIFF = A::NO_DIFF && B::NO_DIFF;
    /* the intersection is empty, or ends before EPS, when every primitive
     * span below A is strictly separated from every one below B or one of
     * the two ends before EPS (with no Difference below, A's and B's output
     * spans lie inside the union of their primitives' spans) */
    template <class PS>
    __device__ static __forceinline__ int isect_empty(const PS &ps)
    {
        int ok = A::isect_empty(ps) & B::isect_empty(ps);
        A::template each_sel<AllPrims>([&](auto x, auto) {
            B::template each_sel<AllPrims>([&](auto y, auto) {
                constexpr int X = decltype(x)::value, Y = decltype(y)::value;
                ok &= sep(ps, X, Y) | inert(ps, X) | inert(ps, Y);
            });
        });
        return ok;
    }
    PTD_BINARY_COMMON
    template <class SEL>
    __device__ static constexpr bool clear_ok() { return A::template nsel<SEL>() + B::template nsel<SEL>() == 0; }
    template <class F>
    __device__ static __forceinline__ void each_pos(F &&) {}
#if PT_PULL_SELECT
    __device__ static __forceinline__ bool pull(St &s, CS &out)
    {
        for (;;) {
            if (s.ea || s.eb)
                return false;
            const float a0 = s.sa.t0, a1 = s.sa.t1, b0 = s.sb.t0, b1 = s.sb.t1;
            const bool skipA = a1 < b0, skipB = !skipA && b1 < a0, over = !skipA && !skipB;
            /* overlap: the later start (start_from_start) and the earlier end;
             * the span whose end is taken is advanced */
            const bool bLater = over && a0 < b0;
            const bool endA = over && (bLater ? a1 < b1 : !(b1 < a1));
            out.t0 = bLater ? b0 : a0, out.r0 = bLater ? s.sb.r0 : s.sa.r0;
            out.t1 = endA ? a1 : b1, out.r1 = endA ? s.sa.r1 : s.sb.r1;
            const bool adv_a = skipA || endA;
            if (adv_a)
                s.ea = !A::pull(s.a, s.sa);
            else
                s.eb = !B::pull(s.b, s.sb);
            if (over)
                return true;
        }
    }
#else
    __device__ static __forceinline__ bool pull(St &s, CS &out)
    {
        for (;;) {
            if (s.ea || s.eb)
                return false;
            bool emit = true, adv_a;
            if (s.sa.t1 < s.sb.t0) {
                emit = false, adv_a = true;
            } else if (s.sb.t1 < s.sa.t0) {
                emit = false, adv_a = false;
            } else if (s.sa.t0 < s.sb.t0) {
                if (s.sa.t1 < s.sb.t1) {
                    start_from_start(s.sa, s.sb);
                    out = s.sa, adv_a = true;
                } else {
                    out = s.sb, adv_a = false;
                }
            } else if (s.sb.t1 < s.sa.t1) {
                start_from_start(s.sb, s.sa);
                out = s.sb, adv_a = false;
            } else {
                out = s.sa, adv_a = true;
            }
            if (adv_a)
                s.ea = !A::pull(s.a, s.sa);
            else
                s.eb = !B::pull(s.b, s.sb);
            if (emit)
                return true;
        }
    }
#endif
};

/* src/difference.cpp:84-135, including the :124-130 copyEndFromStart quirk */
template <class A, class B>
struct Diff
{
    static constexpr int KIND = NODE_DIFF;
    static constexpr bool UNION_ONLY = false;
    static constexpr bool NO_DIFF = false;
    template <class PS>
    __device__ static __forceinline__ int isect_empty(const PS &) { return 0; }
    PTD_BINARY_COMMON
    template <class SEL>
    __device__ static constexpr bool clear_ok() { return A::template nsel<SEL>() + B::template nsel<SEL>() == 0; }
    template <class F>
    __device__ static __forceinline__ void each_pos(F &&f) { A::each_pos(f); }
#if PT_PULL_SELECT
    __device__ static __forceinline__ bool pull(St &s, CS &out)
    {
        for (;;) {
            if (s.ea)
                return false;
            const bool eb = s.eb;
            const float a0 = s.sa.t0, a1 = s.sa.t1, b0 = s.sb.t0, b1 = s.sb.t1;
            const u32 ra0 = s.sa.r0, ra1 = s.sa.r1, rb0 = s.sb.r0, rb1 = s.sb.r1;
            const bool passA = eb || a1 < b0;                     /* A emitted whole           */
            const bool skipB = !passA && b1 < a0;                 /* B before A: next B        */
            const bool over = !passA && !skipB;
            const bool cut = over && a0 < b0;                     /* A emitted up to B's start */
            const bool cutEnd = cut && a1 < b1;                   /*   ... and A is done       */
            const bool cutSplit = cut && !(a1 < b1);              /*   ... A resumes after B   */
            const bool quirk = over && !cut && a1 > b1;           /* :124-130, copyEndFromStart */
            const bool emit = passA || cut;
            const bool adv_a = passA || cutEnd || (over && !cut && !quirk);
            /* emitted span: A's start, and A's end or B's start (flipped) */
            out.t0 = a0, out.r0 = ra0;
            out.t1 = cut ? b0 : a1, out.r1 = cut ? rb0 ^ FLIP : ra1;
            /* A's state when it stays: resumes at B's end (start_from_end), or
             * the quirk's end from B's start (end_from_start) */
            s.sa.t0 = cutSplit ? b1 : a0, s.sa.r0 = cutSplit ? rb1 ^ FLIP : ra0;
            s.sa.t1 = quirk ? b0 : a1, s.sa.r1 = quirk ? rb0 ^ FLIP : ra1;
            if (adv_a)
                s.ea = !A::pull(s.a, s.sa);
            else
                s.eb = !B::pull(s.b, s.sb);
            if (emit)
                return true;
        }
    }
#else
    __device__ static __forceinline__ bool pull(St &s, CS &out)
    {
        for (;;) {
            if (s.ea)
                return false;
            bool emit = true, adv_a = true;
            if (s.eb) {
                out = s.sa;
            } else if (s.sa.t1 < s.sb.t0) {
                out = s.sa;
            } else if (s.sb.t1 < s.sa.t0) {
                emit = false, adv_a = false;
            } else if (s.sa.t0 < s.sb.t0) {
                if (s.sa.t1 < s.sb.t1) {
                    end_from_start(s.sa, s.sb);
                    out = s.sa;
                } else {
                    out = s.sa;
                    end_from_start(out, s.sb);
                    start_from_end(s.sa, s.sb);
                    adv_a = false;
                }
            } else if (s.sa.t1 > s.sb.t1) {
                end_from_start(s.sa, s.sb);
                emit = false, adv_a = false;
            } else {
                emit = false;
            }
            if (adv_a)
                s.ea = !A::pull(s.a, s.sa);
            else
                s.eb = !B::pull(s.b, s.sb);
            if (emit)
                return true;
        }
    }
#endif
};

/* TransformedObject (include/object.h:26-76): the child sees the ray mapped by
 * m; span normals are mapped back by normalize(inv.applyNoTranslate(n)).
 * P[MOFF..+12] = m, P[IOFF..+12] = inverse(m) (transform.h:350-383, host). */
/* ---- union-only passes with the sphere roots compacted per lane ----------
 * (PT_SPH_COMPACT) A fast pass over a tree of Unions, spheres and planes takes
 * the union rule (union_first_hit) as an accumulation whose result does not
 * depend on the order the spans arrive in (the minimum start, a tie on it,
 * a NaN anywhere).  So the spheres' roots and quotients need not run sphere
 * by sphere on the whole wave whenever one lane meets the sphere: each lane
 * first marks the spheres it meets (the discriminant alone), then every lane
 * walks its own marked spheres, reading their contexts from an LDS table by
 * primitive index -- the wave loops as many times as its lanes' largest
 * count, not once per sphere any lane meets. */
#ifndef PT_SPH_COMPACT
#define PT_SPH_COMPACT 1
#endif
struct UnionAcc
{
    int found = 0, tie = 0, bad = 0, bm = 0;
    float b0 = 0.0f;
    __device__ __forceinline__ void add(int live, float t0, float t1, int m)
    {
        const int cand = live & (t1 >= EPS);
        const int better = cand & ((!found) | (t0 < b0));
        tie = better ? 0 : (tie | (cand & (t0 == b0)));
        bad |= live & ((t0 != t0) | (t1 != t1));
        b0 = better ? t0 : b0;
        bm = better ? m : bm;
        found |= cand;
    }
};
/* Opposite unit-normal planes of one axis taken as a pair (PT_PLANE_PAIR):
 * with the origin outside both solids (num <= -eps^2, burst-uniform), a lane
 * moving along -e_k enters only the n_k = +1 plane and leaves the other, whose
 * span [-max_value, t < 0] (or a dead one) is no candidate, no tie, no NaN for
 * the union rule -- so one quotient per lane, of the plane it enters, gives
 * the same accumulation as both.  Compact<Pln>::run parks the first such
 * plane of each (axis, side) here; compact_first_hit evaluates the parked
 * ones once the tree is walked (a pair when both sides are parked). */
#ifndef PT_PLANE_PAIR
#define PT_PLANE_PAIR 1
#endif
struct PlaneStash
{
    float num[3][2];
    int mat[3][2];
    int has[3][2];
};
template <class N>
struct Compact
{
    static constexpr bool OK = false;
};
template <int P, int O, int M>
struct Compact<Sph<P, O, M>>
{
    static constexpr bool OK = P < 64;
    __device__ static __forceinline__ void run(UnionAcc &, u64 &m, PlaneStash &,
                                               const typename Sph<P, O, M>::Ctx &c, const Ray &q, const Env &)
    {
        const float b = dot(c.omc, q.d);
        const float disc = b * b - q.a * c.c;
        if (!(disc <= EPS))
            m |= 1ull << P;
    }
    __device__ static __forceinline__ void fill(float4 *tab, int *mt, const typename Sph<P, O, M>::Ctx &c)
    {
        tab[P] = make_float4(c.omc.x, c.omc.y, c.omc.z, c.c);
        mt[P] = M;
    }
};
template <int P, int O, int M, int AX, int U>
struct Compact<Pln<P, O, M, AX, U>>
{
    static constexpr bool OK = true;
    __device__ static __forceinline__ void run(UnionAcc &acc, u64 &, PlaneStash &st,
                                               const typename Pln<P, O, M, AX, U>::Ctx &c, const Ray &q, const Env &e)
    {
#if defined(PT_AXIS_SHARE) && PT_PLANE_PAIR
        if constexpr (U != 0 && AX >= 0) {
            constexpr int k = AX >> 1, side = AX & 1;
            if (c.num <= -(EPS * EPS) && !st.has[k][side]) {
                st.num[k][side] = c.num, st.mat[k][side] = M, st.has[k][side] = 1;
                return;
            }
        }
#endif
        typename Pln<P, O, M, AX, U>::St s;
        Pln<P, O, M, AX, U>::init(s, c, q, e);
        acc.add(s.live, s.t0, s.t1, M);
    }
    __device__ static __forceinline__ void fill(float4 *, int *, const typename Pln<P, O, M, AX, U>::Ctx &) {}
};
template <class A, class B>
struct Compact<Uni<A, B>>
{
    static constexpr bool OK = Compact<A>::OK && Compact<B>::OK;
    __device__ static __forceinline__ void run(UnionAcc &acc, u64 &m, PlaneStash &st, const typename Uni<A, B>::Ctx &c,
                                               const Ray &q, const Env &e)
    {
        Compact<A>::run(acc, m, st, c.a, q, e);
        Compact<B>::run(acc, m, st, c.b, q, e);
    }
    __device__ static __forceinline__ void fill(float4 *tab, int *mt, const typename Uni<A, B>::Ctx &c)
    {
        Compact<A>::fill(tab, mt, c.a);
        Compact<B>::fill(tab, mt, c.b);
    }
};
/* union_first_hit's result for a Compact tree: planes in line, the marked
 * spheres walked per lane from the table */
template <class R>
__device__ __forceinline__ int compact_first_hit(const typename R::Ctx &ctx, const Ray &q, const Env &e,
                                                 const float4 *tab, const int *mt, bool &hit, float &t, int &mat)
{
    UnionAcc acc;
    u64 m = 0ull;
    PlaneStash st;
#pragma unroll
    for (int k = 0; k < 3; k++)
        st.has[k][0] = st.has[k][1] = 0;
    Compact<R>::run(acc, m, st, ctx, q, e);
#if defined(PT_AXIS_SHARE) && PT_PLANE_PAIR
    /* the parked unit planes: Pln::init's UNIT arithmetic on the plane each
     * lane enters (n_k = +1 when d_k < 0), or on each parked plane alone */
    auto unit_plane = [&](int k, int side, float num, int mat) {
        const float dk = k == 0 ? q.d.x : k == 1 ? q.d.y : q.d.z;
        const float div = side ? -dk : dk; /* n_k d_k, n_k = +-1 exactly */
        const bool small = __builtin_fabsf(div) < EPS * EPS;
        const float q0 = div_core(num, q.rk[k]);
        float t = side ? -q0 : q0;
        const bool bad = !small && !(q.rkok[k] && num_ok(num));
        if (wave_any(bad)) {
            if (bad)
                t = num / div;
        }
        const bool deg = small || __builtin_fabsf(t) >= MAXV;
        const bool neg = div < 0.0f;
        acc.add((!deg || __builtin_fabsf(num) < EPS * EPS) ? 1 : 0, (!deg && neg) ? t : -MAXV,
                (!deg && !neg) ? t : MAXV, mat);
    };
#pragma unroll
    for (int k = 0; k < 3; k++) {
        if (st.has[k][0] && st.has[k][1]) {
            const float dk = k == 0 ? q.d.x : k == 1 ? q.d.y : q.d.z;
            const int side = dk < 0.0f ? 0 : 1;
            unit_plane(k, side, side ? st.num[k][1] : st.num[k][0], side ? st.mat[k][1] : st.mat[k][0]);
        } else {
            if (st.has[k][0])
                unit_plane(k, 0, st.num[k][0], st.mat[k][0]);
            if (st.has[k][1])
                unit_plane(k, 1, st.num[k][1], st.mat[k][1]);
        }
    }
#endif
    while (wave_any(m != 0ull)) {
        if (m != 0ull) {
            const int k = __builtin_ctzll(m);
            m &= m - 1ull;
            const float4 sp = tab[k];
            const float b = (sp.x * q.d.x + sp.y * q.d.y) + sp.z * q.d.z; /* dot(omc, d), Sph::init */
            const float disc = b * b - q.a * sp.w;
            const float sq = sqrt_core(disc); /* exact: disc > EPS (or inf / NaN) on a marked sphere */
            const float n0 = -b - sq, n1 = -b + sq;
            float t0 = div_core(n0, q.ra), t1 = div_core(n1, q.ra);
            if (!(q.aok && num_ok(n0) && num_ok(n1)))
                t0 = n0 / q.a, t1 = n1 / q.a;
            acc.add(1, t0, t1, mt[k]);
        }
    }
    mat = acc.bm;
    t = acc.b0;
    hit = acc.found && acc.b0 < MAXV;
    return ((!acc.found) | ((acc.b0 >= EPS) & !acc.tie)) & !acc.bad;
}

/* ---- leaf children occluded by a plane (PT_OCCLUDE) ----------------------
 * In a tree of Unions, spheres and planes the first hit of a ray is the
 * earliest merged span (src/union.cpp:84-134): its start material when the
 * start reaches eps, else nothing when it runs to max_value
 * (path-trace.h:66-96).  A non-emissive plane whose solid the child ray
 * enters at t_P (origin outside, d.n < 0) gives the span [t_P, max_value],
 * so the merged span holding it, and every span before it, starts at or
 * before t_P.  If every emissive primitive's span starts after t_P, the hit
 * is non-emissive or none: the child's term is weight * (+0, +0, +0), zero
 * for the finite weights RAW already requires, like a dark child's.
 * T_E, a lower bound on the emissive starts from the burst origin, is taken
 * once per burst: an emissive plane the origin is outside of (num <= -1e-3)
 * cannot be met before |num| / |n| (less 0.1 % for the rounding of the
 * computed quotient); an emissive sphere, or an origin inside an emissive
 * plane's solid, gives T_E = 0 (no claim).  Per attempt, on the
 * unnormalised w with |w| <= B = (1 + |kR|) 1.0001 (accepted: |v| < 1), an
 * axis-aligned occluder (the exact n.w = n_a w_a) is entered before T_E when
 * n_a w_a < -|num_P| B 1.001 / T_E: the normalised direction's quotient is
 * then at most T_E (1 + 3e-6) / 1.001.  The occluder needs |n_a w_a| > 1e-4
 * (a non-degenerate span) and num_P <= -1e-3. */
#ifndef PT_OCCLUDE
#define PT_OCCLUDE 1
#endif
template <class N>
struct Occl
{
    static constexpr bool OK = false;
};
template <int P, int O, int M>
struct Occl<Sph<P, O, M>>
{
    static constexpr bool OK = true;
    template <class SEL>
    __device__ static __forceinline__ float emis_lb(const typename Sph<P, O, M>::Ctx &, const Env &)
    {
        return SEL::take(M) ? 0.0f : __builtin_inff();
    }
    template <class SEL>
    __device__ static __forceinline__ u64 occ(const typename Sph<P, O, M>::Ctx &, V3, float, const Env &)
    {
        return 0ull;
    }
};
template <int P, int O, int M, int AX, int U>
struct Occl<Pln<P, O, M, AX, U>>
{
    static constexpr bool OK = true;
    template <class SEL>
    __device__ static __forceinline__ float emis_lb(const typename Pln<P, O, M, AX, U>::Ctx &c, const Env &e)
    {
        if constexpr (!SEL::take(M))
            return __builtin_inff();
        const float nn = __builtin_sqrtf(dot(mk(e.P[O], e.P[O + 1], e.P[O + 2]), mk(e.P[O], e.P[O + 1], e.P[O + 2])));
        return c.num <= -1e-3f ? (-c.num / nn) * 0.999f : 0.0f;
    }
    template <class SEL>
    __device__ static __forceinline__ u64 occ(const typename Pln<P, O, M, AX, U>::Ctx &c, V3 w, float g, const Env &e)
    {
        if constexpr (SEL::take(M) || AX < 0) {
            return 0ull;
        } else {
            const float na = e.P[O + (AX >> 1)];
            const float wa = (AX >> 1) == 0 ? w.x : (AX >> 1) == 1 ? w.y : w.z;
            const float lim = fmaxf(1e-4f, -c.num * g);
            return __ballot(c.num <= -1e-3f && na * wa < -lim);
        }
    }
};
template <class A, class B>
struct Occl<Uni<A, B>>
{
    static constexpr bool OK = Occl<A>::OK && Occl<B>::OK;
    template <class SEL>
    __device__ static __forceinline__ float emis_lb(const typename Uni<A, B>::Ctx &c, const Env &e)
    {
        return fminf(Occl<A>::template emis_lb<SEL>(c.a, e), Occl<B>::template emis_lb<SEL>(c.b, e));
    }
    template <class SEL>
    __device__ static __forceinline__ u64 occ(const typename Uni<A, B>::Ctx &c, V3 w, float g, const Env &e)
    {
        return Occl<A>::template occ<SEL>(c.a, w, g, e) | Occl<B>::template occ<SEL>(c.b, w, g, e);
    }
};

template <int MOFF, int IOFF, class C>
struct Xf
{
    static constexpr int LO = C::LO, HI = C::HI;
    static constexpr bool UNION_ONLY = C::UNION_ONLY; /* spans keep the ray's t */
    static constexpr bool NO_DIFF = C::NO_DIFF;
    template <class PS>
    __device__ static __forceinline__ int isect_empty(const PS &ps) { return C::isect_empty(ps); }
    struct Ctx
    {
        typename C::Ctx c;
    };
    typedef typename C::St St;
    __device__ static __forceinline__ void prep(Ctx &c, V3 o, const Env &e) { C::prep(c.c, univ(m_apply(e.P + MOFF, o)), e); }
    __device__ static __forceinline__ void prep_l(Ctx &c, V3 o, const Env &e) { C::prep_l(c.c, m_apply(e.P + MOFF, o), e); }
    __device__ static __forceinline__ void init(St &s, const Ctx &c, const Ray &q, const Env &e)
    {
        C::init(s, c.c, mkray(m_lin(e.P + MOFF, q.d)), e);
    }
    __device__ static __forceinline__ bool pull(St &s, CS &out) { return C::pull(s, out); }
    template <class PS>
    __device__ static __forceinline__ void span(PS &ps, const Ctx &c, const Ray &q, const Env &e)
    {
        C::span(ps, c.c, mkray(m_lin(e.P + MOFF, q.d)), e);
    }
    template <class PS>
    __device__ static __forceinline__ void init_ps(St &s, const PS &ps) { C::init_ps(s, ps); }
    template <class F>
    __device__ static __forceinline__ void each_pos(F &&f) { C::each_pos(f); }
    template <class SEL, class PS>
    __device__ static __forceinline__ void span_sel(PS &ps, const Ctx &c, const Ray &q, const Env &e)
    {
        C::template span_sel<SEL>(ps, c.c, mkray(m_lin(e.P + MOFF, q.d)), e);
    }
    template <class SEL, class F>
    __device__ static __forceinline__ void each_sel(F &&f) { C::template each_sel<SEL>(f); }
    /* the transformed direction is not normalised: spheres inside use the
     * origin-outside rule only */
    template <class SEL, bool NORM>
    __device__ static __forceinline__ u64 clear_mask(const Ctx &c, const Ray &q, const Env &e)
    {
        return C::template clear_mask<SEL, false>(c.c, mkray(m_lin(e.P + MOFF, q.d)), e);
    }
    template <class SEL>
    __device__ static constexpr bool clear_ok() { return C::template clear_ok<SEL>(); }
    template <class PS>
    __device__ static __forceinline__ int fast_ok(const PS &ps) { return C::fast_ok(ps); }
    __device__ static __forceinline__ V3 normal(int prim, float t, V3 o, V3 d, const Env &e)
    {
        V3 n = C::normal(prim, t, m_apply(e.P + MOFF, o), m_lin(e.P + MOFF, d), e);
        return PT_NORM(m_lin(e.P + IOFF, n));
    }
    /* no raw-direction dark test through a transform unless nothing inside is selected */
    template <class SEL>
    __device__ static constexpr bool raw_ok() { return C::template nsel<SEL>() == 0; }
    template <class SEL>
    __device__ static constexpr int nsel() { return C::template nsel<SEL>(); }
    template <class SEL>
    __device__ static __forceinline__ u64 dark_mask(const Ctx &, V3, const Env &) { return ~0ull; }
    template <class SEL>
    __device__ static __forceinline__ bool dark_pre(const Ctx &, const Env &) { return true; }
};

/* First qualifying span of the root, traceRay's scan (path-trace.h:66-100). */
template <class R>
__device__ __forceinline__ bool first_hit(const typename R::Ctx &ctx, V3 d, const Env &e, float &t, u32 &ref,
                                          bool &exit_hit)
{
#ifdef PT_MERGE_STUB /* diagnostic builds only: every lazy merge left out (wrong bits) */
    (void)ctx, (void)d, (void)e, (void)t, (void)ref, (void)exit_hit;
    return false;
#endif
    typename R::St st;
    R::init(st, ctx, mkray(d), e);
    CS s;
    while (R::pull(st, s)) {
        if (s.t0 >= MAXV)
            return false;
        if (s.t0 >= EPS) {
            t = s.t0, ref = s.r0, exit_hit = false;
            return true;
        }
        if (s.t1 >= MAXV)
            return false;
        if (s.t1 >= EPS) {
            t = s.t1, ref = s.r1, exit_hit = true;
            return true;
        }
    }
    return false;
}

/* The same lazy merge started from the primitive spans the fast checks just
 * computed (init_ps: the values init() would compute): the primitive contexts
 * are dead by then and the spans are not computed twice. */
template <class R, class PS>
__device__ __forceinline__ bool first_hit_ps(const PS &ps, float &t, u32 &ref, bool &exit_hit)
{
    typename R::St st;
    R::init_ps(st, ps);
    CS s;
    while (R::pull(st, s)) {
        if (s.t0 >= MAXV)
            return false;
        if (s.t0 >= EPS) {
            t = s.t0, ref = s.r0, exit_hit = false;
            return true;
        }
        if (s.t1 >= MAXV)
            return false;
        if (s.t1 >= EPS) {
            t = s.t1, ref = s.r1, exit_hit = true;
            return true;
        }
    }
    return false;
}

/* First hit from every primitive's span at once, where the fast checks hold
 * (the union rule in union-only trees, else the pairwise checks): the hit is
 * then a positive primitive's own boundary -- its start (entry) if that is
 * >= EPS, else its end (exit, the pairs around it strictly separated), never
 * a flipped one -- so the reference's ref and exit flag follow from the
 * chosen primitive.  Returns the check's verdict; the result is valid only
 * where it holds. */
template <class R, class PS>
__device__ __forceinline__ int cheap_ok(const PS &ps);
template <class R, class PS>
__device__ __forceinline__ int span_first_hit(const PS &ps, bool &hit, float &t, u32 &ref, bool &exit_hit)
{
    int fok;
    if constexpr (R::NO_DIFF) {
        /* one pass over the spans; the pairwise checks only where it cannot decide */
        fok = cheap_ok<R>(ps);
        if (wave_any(!fok)) {
            if (!fok)
                fok = R::fast_ok(ps);
        }
    } else {
        fok = R::fast_ok(ps);
    }
    int found = 0;
    u32 bref = 0u;
    float b0 = 0.0f, b1 = 0.0f;
    R::each_pos([&](auto x, auto m) {
        constexpr int X = decltype(x)::value;
        const int cand = ps.live[X] & (ps.t1[X] >= EPS);
        const int better = cand & ((!found) | (ps.t0[X] < b0));
        b0 = better ? ps.t0[X] : b0;
        b1 = better ? ps.t1[X] : b1;
        bref = better ? mkref(X, decltype(m)::value, 0) : bref;
        found |= cand;
    });
    hit = false;
    if (found && b0 < MAXV) {
        if (b0 >= EPS)
            hit = true, t = b0, ref = bref, exit_hit = false;
        else if (b1 < MAXV)
            hit = true, t = b1, ref = bref | 2u, exit_hit = true; /* mkref(prim, mat, 1) */
    }
    return fok;
}

/* Spine and lane queries start the lazy merge from the spans they computed */
#ifndef PT_MERGE_FROM_SPANS
#define PT_MERGE_FROM_SPANS 1
#endif
/* The spine's query (one ray, the same on every lane): span_first_hit where
 * the checks hold, else the lazy merge.  The checks are wave-uniform here. */
template <class R>
__device__ __forceinline__ bool spine_first_hit(const typename R::Ctx &ctx, V3 d, const Env &e, float &t, u32 &ref,
                                                bool &exit_hit, int &merged)
{
    PrimSpans<R::HI> ps;
    R::span(ps, ctx, mkray(d), e);
    bool hit;
    const int fok = span_first_hit<R>(ps, hit, t, ref, exit_hit);
    merged = 0;
    if (!wave_any(!fok))
        return hit;
    merged = 1;
#if PT_MERGE_FROM_SPANS
    (void)ctx, (void)d, (void)e;
    return first_hit_ps<R>(ps, t, ref, exit_hit);
#else
    return first_hit<R>(ctx, d, e, t, ref, exit_hit);
#endif
}

#ifdef PT_BAIL_STATS /* diagnostic builds: which chunks a merge-free kernel could finish */
__device__ unsigned pt_bail_flag[1 << 20];
__device__ __forceinline__ void pt_bail_mark() { pt_bail_flag[blockIdx.x * blockDim.x + threadIdx.x] = 1u; }
#endif
/* A lane's own query (camera rays, lane-finished mirror children): the same,
 * the lazy merge only on the lanes whose checks fail. */
template <class R>
__device__ __forceinline__ bool lane_first_hit(const typename R::Ctx &ctx, V3 d, const Env &e, float &t, u32 &ref,
                                               bool &exit_hit)
{
#if defined(PT_FAST_SPINE) || defined(PT_FAST_LANE)
    PrimSpans<R::HI> ps;
    R::span(ps, ctx, mkray(d), e);
    bool hit;
    const int fok = span_first_hit<R>(ps, hit, t, ref, exit_hit);
    if (wave_any(!fok)) {
#ifdef PT_BAIL_STATS
        if (!fok)
            pt_bail_mark();
#endif
        if (!fok)
#if PT_MERGE_FROM_SPANS
            hit = first_hit_ps<R>(ps, t, ref, exit_hit);
#else
            hit = first_hit<R>(ctx, d, e, t, ref, exit_hit);
#endif
    }
    return hit;
#else
    return first_hit<R>(ctx, d, e, t, ref, exit_hit);
#endif
}

/* The light kernel's lane query (split launches): the fast checks alone.
 * undecided = the checks failed on this lane, whose sample then goes to the
 * full kernel with its whole chunk (t / ref are not valid then). */
template <class R>
__device__ __forceinline__ bool lane_first_hit_light(const typename R::Ctx &ctx, V3 d, const Env &e, float &t,
                                                     u32 &ref, bool &exit_hit, bool &undecided)
{
    PrimSpans<R::HI> ps;
    R::span(ps, ctx, mkray(d), e);
    bool hit;
    undecided = !span_first_hit<R>(ps, hit, t, ref, exit_hit);
    return hit && !undecided;
}

/* Fast first hit over precomputed primitive spans; valid when R::fast_ok. */
template <class R, class PS>
__device__ __forceinline__ bool fast_first_hit(const PS &ps, float &t, int &mat)
{
    int found = 0, bm = 0;
    float b0 = 0.0f, b1 = 0.0f;
    R::each_pos([&](auto x, auto m) {
        constexpr int X = decltype(x)::value;
        const int cand = ps.live[X] & (ps.t1[X] >= EPS);
        const int better = cand & ((!found) | (ps.t0[X] < b0));
        b0 = better ? ps.t0[X] : b0;
        b1 = better ? ps.t1[X] : b1;
        bm = better ? decltype(m)::value : bm;
        found |= cand;
    });
    mat = bm;
    if (!found || b0 >= MAXV)
        return false;
    if (b0 >= EPS) {
        t = b0;
        return true;
    }
    if (b1 >= MAXV)
        return false;
    t = b1;
    return true;
}

/* Union merges (src/union.cpp:84-134) turn the spans below a node into the
 * connected components of their union (overlapping or touching spans merge,
 * the smaller start kept).  So where only Unions (and transforms, which keep
 * the ray's t) combine a set of primitives, and b0 -- the smallest start among
 * their live spans reaching EPS -- is itself >= EPS and no other such span
 * starts at b0, the first component reaching EPS starts at b0: a span ending
 * before EPS cannot touch it and every other span reaching EPS starts later.
 * traceRay's scan (path-trace.h:66-100) stops there, at fast_first_hit's /
 * sel_first_hit's answer, however the spans overlap: one pass over the spans
 * instead of the pairwise separation checks.  No candidate at all: nothing is
 * hit.  NaN bounds never pass. */
template <class PS, class EACH>
__device__ __forceinline__ int union_min_ok(const PS &ps, EACH &&each)
{
    int found = 0, tie = 0, bad = 0;
    float b0 = 0.0f;
    each([&](auto x, auto) {
        constexpr int X = decltype(x)::value;
        const int live = ps.live[X];
        const int cand = live & (ps.t1[X] >= EPS);
        const int better = cand & ((!found) | (ps.t0[X] < b0));
        tie = better ? 0 : (tie | (cand & (ps.t0[X] == b0)));
        bad |= live & ((ps.t0[X] != ps.t0[X]) | (ps.t1[X] != ps.t1[X]));
        b0 = better ? ps.t0[X] : b0;
        found |= cand;
    });
    return ((!found) | ((b0 >= EPS) & !tie)) & !bad;
}

/* The one-pass check of a tree without Difference nodes: its Intersections
 * are empty or end before EPS (isect_empty), so only Unions and transforms
 * combine what can be met at or after EPS -- the union rule over the
 * positive primitives (each_pos leaves Intersection subtrees out). */
template <class R, class PS>
__device__ __forceinline__ int cheap_ok(const PS &ps)
{
    static_assert(R::NO_DIFF, "cheap_ok needs a tree without Difference nodes");
    const int u = union_min_ok(ps, [&](auto &&f) { R::each_pos(f); });
    if constexpr (R::UNION_ONLY)
        return u;
    else
        return u & R::isect_empty(ps);
}

/* cheap_ok and fast_first_hit of a union-only tree in one pass over the
 * spans (the same candidate / better / minimum chain serves both): where the
 * union rule holds and a candidate exists its start b0 is >= EPS, so the hit
 * is that primitive's entry at b0 unless b0 >= MAXV -- fast_first_hit's exit
 * branch (b0 < EPS) cannot occur.  Returns the rule's verdict; hit / t / mat
 * are valid where it holds. */
#ifndef PT_UNION_FUSED
#define PT_UNION_FUSED 1
#endif
template <class R, class PS>
__device__ __forceinline__ int union_first_hit(const PS &ps, bool &hit, float &t, int &mat)
{
    static_assert(R::UNION_ONLY, "union_first_hit needs a union-only tree");
    int found = 0, tie = 0, bad = 0, bm = 0;
    float b0 = 0.0f;
    R::each_pos([&](auto x, auto m) {
        constexpr int X = decltype(x)::value;
        const int live = ps.live[X];
        const int cand = live & (ps.t1[X] >= EPS);
        const int better = cand & ((!found) | (ps.t0[X] < b0));
        tie = better ? 0 : (tie | (cand & (ps.t0[X] == b0)));
        bad |= live & ((ps.t0[X] != ps.t0[X]) | (ps.t1[X] != ps.t1[X]));
        b0 = better ? ps.t0[X] : b0;
        bm = better ? decltype(m)::value : bm;
        found |= cand;
    });
    mat = bm;
    t = b0;
    hit = found && b0 < MAXV;
    return ((!found) | ((b0 >= EPS) & !tie)) & !bad;
}

/* ---- clear pass -------------------------------------
 * When every selected (emissive) primitive is reached from the root through
 * Union and TransformedObject nodes only (R::clear_ok), and on a lane every
 * other primitive's span is dead or ends before EPS (R::clear_mask), the
 * lazy merges cannot move the first qualifying span away from the selected
 * primitives' own: a Difference or Intersection subtree then holds no
 * selected primitive, so each span it emits starts and ends at boundaries of
 * its own spans (src/difference.cpp:84-135, src/intersection.cpp:84-130,
 * including the :124-130 quirk's inverted spans) and ends before EPS; at a
 * Union (src/union.cpp:84-134) such a span either lies strictly before a
 * selected span that starts at >= EPS, or merges with one that starts before
 * EPS into a span starting before EPS and ending at that span's own end (the
 * larger end, with its normal) -- the scan (path-trace.h:66-100) skips the
 * former and stops at that same end in the latter.  So the first hit is
 * fast_first_hit over the selected primitives alone, checked pairwise like
 * the fast pass (pair_ok at a Union) when there are several. */
template <class R, class SEL, class PS>
__device__ __forceinline__ int sel_pairs_ok(const PS &ps);
/* The clear pass's check over the selected primitives: with two or more, the
 * union rule above first (they hang off the root through Unions and
 * transforms only, and every other span ends before EPS), the pairwise checks
 * only on the lanes it cannot decide. */
template <class R, class SEL, class PS>
__device__ __forceinline__ int sel_ok(const PS &ps)
{
    if constexpr (R::template nsel<SEL>() < 2) {
        return sel_pairs_ok<R, SEL>(ps);
    } else {
        int ok = union_min_ok(ps, [&](auto &&f) { R::template each_sel<SEL>(f); });
        if (wave_any(!ok)) {
            if (!ok)
                ok = sel_pairs_ok<R, SEL>(ps);
        }
        return ok;
    }
}
template <class R, class SEL, class PS>
__device__ __forceinline__ int sel_pairs_ok(const PS &ps)
{
    int ok = 1;
    R::template each_sel<SEL>([&](auto x, auto) {
        R::template each_sel<SEL>([&](auto y, auto) {
            if constexpr (decltype(x)::value < decltype(y)::value)
                ok &= pair_ok<NODE_UNION>(ps, decltype(x)::value, decltype(y)::value);
        });
    });
    return ok;
}
template <class R, class SEL, class PS>
__device__ __forceinline__ bool sel_first_hit(const PS &ps, float &t, int &mat)
{
    int found = 0, bm = 0;
    float b0 = 0.0f, b1 = 0.0f;
    R::template each_sel<SEL>([&](auto x, auto m) {
        constexpr int X = decltype(x)::value;
        const int cand = ps.live[X] & (ps.t1[X] >= EPS);
        const int better = cand & ((!found) | (ps.t0[X] < b0));
        b0 = better ? ps.t0[X] : b0;
        b1 = better ? ps.t1[X] : b1;
        bm = better ? decltype(m)::value : bm;
        found |= cand;
    });
    mat = bm;
    if (!found || b0 >= MAXV)
        return false;
    if (b0 >= EPS) {
        t = b0;
        return true;
    }
    if (b1 >= MAXV)
        return false;
    t = b1;
    return true;
}

/* Selects the primitives whose material may emit (scene S::dark is false). */
template <class S>
struct Emissive
{
    __device__ static constexpr bool take(int m) { return !S::dark(m); }
};

/* ------------------------------------------------------------ textures --- */
__device__ __forceinline__ float mean3(V3 c) { return ((c.x + c.y) + c.z) * (1.0f / 3.0f); } /* texture.h:14-18 */

__device__ __forceinline__ V3 img_rgb(const PtImage &im, int x, int y)
{
    if (!im.data || y < 0 || (u32)y >= im.h || x < 0 || (u32)x >= im.w)
        return mk(0, 0, 0);
    float4 v = im.data[(u32)x + (u32)y * im.w];
    return mk(v.x, v.y, v.z);
}
__device__ __forceinline__ float img_alpha(const PtImage &im, int x, int y)
{
    if (!im.data || y < 0 || (u32)y >= im.h || x < 0 || (u32)x >= im.w)
        return 0.0f;
    return im.data[(u32)x + (u32)y * im.w].w;
}
/* ImageTexture texel (image_texture.h:20-27): `x -= floor(x)` runs in double */
__device__ __forceinline__ void planar_texel(const PtImage &im, V3 v, int &xi, int &yi)
{
    float x = v.x, y = v.y;
    x = (float)((double)x - __builtin_floor((double)x));
    y = (float)((double)y - __builtin_floor((double)y));
    y = 1.0f - y;
    x *= (float)im.w;
    y *= (float)im.h;
    xi = cvt_x86(__builtin_floorf(x));
    yi = cvt_x86(__builtin_floorf(y));
}
__device__ __forceinline__ int skybox_face(V3 v, float &fx, float &fy) /* image_texture.h:94-109 */
{
    V3 a = mk(__builtin_fabsf(v.x), __builtin_fabsf(v.y), __builtin_fabsf(v.z));
    if (a.x > a.y && a.x > a.z) {
        if (v.x < 0.0f) {
            fx = -v.z / a.x, fy = v.y / a.x;
            return 2; /* left */
        }
        fx = v.z / a.x, fy = v.y / a.x;
        return 3; /* right */
    }
    if (a.y > a.z) {
        if (v.y < 0.0f) {
            fx = -v.x / a.y, fy = v.z / a.y;
            return 1; /* bottom */
        }
        fx = v.x / a.y, fy = v.z / a.y;
        return 0; /* top */
    }
    if (v.z < 0.0f) {
        fx = v.x / a.z, fy = v.y / a.z;
        return 5; /* back */
    }
    fx = -v.x / a.z, fy = v.y / a.z;
    return 4; /* front */
}
__device__ __forceinline__ void skybox_texel(const PtImage &im, float x, float y, int &xi, int &yi)
{
    x = (float)((double)x * 0.5 + 0.5);
    y = (float)(0.5 - (double)y * 0.5);
    x *= (float)im.w;
    y *= (float)im.h;
    xi = cvt_x86(__builtin_floorf(x));
    yi = cvt_x86(__builtin_floorf(y));
}

template <int OFF>
struct TConst /* ColorTexture */
{
    __device__ static __forceinline__ V3 color(V3, const Env &e) { return mk(e.P[OFF], e.P[OFF + 1], e.P[OFF + 2]); }
    __device__ static __forceinline__ float value(V3 p, const Env &e) { return mean3(color(p, e)); }
};
struct TCoord /* test instrument */
{
    __device__ static __forceinline__ V3 color(V3 p, const Env &) { return p; }
    __device__ static __forceinline__ float value(V3 p, const Env &e) { return mean3(color(p, e)); }
};
template <int MOFF, class T>
struct TXf /* TransformedTexture */
{
    __device__ static __forceinline__ V3 color(V3 p, const Env &e) { return T::color(m_apply(e.P + MOFF, p), e); }
    __device__ static __forceinline__ float value(V3 p, const Env &e) { return T::value(m_apply(e.P + MOFF, p), e); }
};
template <int SLOT>
struct TImage /* ImageTexture */
{
    __device__ static __forceinline__ V3 color(V3 p, const Env &e)
    {
        int x, y;
        planar_texel(e.img[SLOT], p, x, y);
        return img_rgb(e.img[SLOT], x, y);
    }
    __device__ static __forceinline__ float value(V3 p, const Env &e) { return mean3(color(p, e)); }
};
template <int SLOT>
struct TImageAlpha /* ImageAlphaTexture */
{
    __device__ static __forceinline__ float value(V3 p, const Env &e)
    {
        int x, y;
        planar_texel(e.img[SLOT], p, x, y);
        return img_alpha(e.img[SLOT], x, y);
    }
    __device__ static __forceinline__ V3 color(V3 p, const Env &e)
    {
        float a = value(p, e);
        return mk(a, a, a);
    }
};
template <int S0, int S1, int S2, int S3, int S4, int S5>
struct TSkybox /* ImageSkyboxTexture: top bottom left right front back */
{
    __device__ static __forceinline__ V3 color(V3 v, const Env &e)
    {
        if (is_zero(v))
            return mk(0, 0, 0);
        float fx, fy;
        int f = skybox_face(v, fx, fy);
        const int slots[6] = {S0, S1, S2, S3, S4, S5};
        const PtImage &im = e.img[slots[f]];
        int x, y;
        skybox_texel(im, fx, fy, x, y);
        return img_rgb(im, x, y);
    }
    __device__ static __forceinline__ float value(V3 p, const Env &e) { return mean3(color(p, e)); }
};
template <int S0, int S1, int S2, int S3, int S4, int S5>
struct TSkyboxAlpha /* ImageSkyboxAlphaTexture */
{
    __device__ static __forceinline__ float value(V3 v, const Env &e)
    {
        if (is_zero(v))
            return 0.0f;
        float fx, fy;
        int f = skybox_face(v, fx, fy);
        const int slots[6] = {S0, S1, S2, S3, S4, S5};
        const PtImage &im = e.img[slots[f]];
        int x, y;
        skybox_texel(im, fx, fy, x, y);
        return img_alpha(im, x, y);
    }
    __device__ static __forceinline__ V3 color(V3 v, const Env &e)
    {
        float a = value(v, e);
        return mk(a, a, a);
    }
};
template <int OFF, class T>
struct TMul /* MultiplyTexture */
{
    __device__ static __forceinline__ V3 color(V3 p, const Env &e)
    {
        return T::color(p, e) * mk(e.P[OFF], e.P[OFF + 1], e.P[OFF + 2]);
    }
    __device__ static __forceinline__ float value(V3 p, const Env &e) { return mean3(color(p, e)); }
};
/* The reference's std::log(float) is glibc's logf, which is not correctly
 * rounded: (float)log((double)x) differs from it on 416 909 of the 2^31 - 2^23
 * finite positive floats.  Restated: glibc 2.35's sysdeps/ieee754/flt-32/
 * e_logf.c (Szabolcs Nagy, ARM optimized-routines; MIT/BSD-style licence, see
 * tools/libm/logf_restated.c): a 16-entry table of (1/c, log c), log1p of
 * z/c - 1 by a degree-3 polynomial, all in double.  Checked on the CPU against
 * glibc on every non-negative float, with and without FMA contraction of the
 * double arithmetic (glibc ships FMA variants): no difference
 * (tools/libm/logf_restated.c). */
__device__ __forceinline__ double logf_tab(int i, int hi)
{
    /* (invc, logc) pairs, __logf_data.tab */
    constexpr double T[32] = {
        0x1.661ec79f8f3bep+0, -0x1.57bf7808caadep-2, 0x1.571ed4aaf883dp+0, -0x1.2bef0a7c06ddbp-2,
        0x1.49539f0f010bp+0,  -0x1.01eae7f513a67p-2, 0x1.3c995b0b80385p+0, -0x1.b31d8a68224e9p-3,
        0x1.30d190c8864a5p+0, -0x1.6574f0ac07758p-3, 0x1.25e227b0b8eap+0,  -0x1.1aa2bc79c81p-3,
        0x1.1bb4a4a1a343fp+0, -0x1.a4e76ce8c0e5ep-4, 0x1.12358f08ae5bap+0, -0x1.1973c5a611cccp-4,
        0x1.0953f419900a7p+0, -0x1.252f438e10c1ep-5, 0x1p+0,               0x0p+0,
        0x1.e608cfd9a47acp-1, 0x1.aa5aa5df25984p-5,  0x1.ca4b31f026aap-1,  0x1.c5e53aa362eb4p-4,
        0x1.b2036576afce6p-1, 0x1.526e57720db08p-3,  0x1.9c2d163a1aa2dp-1, 0x1.bc2860d22477p-3,
        0x1.886e6037841edp-1, 0x1.1058bc8a07ee1p-2,  0x1.767dcf5534862p-1, 0x1.4043057b6ee09p-2};
    double r = T[hi];
#pragma unroll
    for (int k = 1; k < 16; k++) /* selects, not a private array indexed per lane */
        r = i == k ? T[2 * k + hi] : r;
    return r;
}
__device__ __forceinline__ float libm_logf(float x)
{
    constexpr double LN2 = 0x1.62e42fefa39efp-1, A0 = -0x1.00ea348b88334p-2, A1 = 0x1.5575b0be00b6ap-2,
                     A2 = -0x1.ffffef20a4123p-2;
    u32 ix = __float_as_uint(x);
    if (ix == 0x3f800000u)
        return 0.0f;
    if (ix - 0x00800000u >= 0x7f800000u - 0x00800000u) {
        if (ix * 2u == 0u)
            return -__builtin_inff();
        if (ix == 0x7f800000u)
            return x;
        if ((ix & 0x80000000u) || ix * 2u >= 0xff000000u)
            return __builtin_nanf("");
        ix = __float_as_uint(x * 0x1p23f); /* subnormal: normalise */
        ix -= 23u << 23;
    }
    const u32 tmp = ix - 0x3f330000u;
    const int i = (int)((tmp >> 19) % 16u), k = (int)tmp >> 23;
    const u32 iz = ix - (tmp & (0x1ffu << 23));
    const double invc = logf_tab(i, 0), logc = logf_tab(i, 1);
    const double z = (double)__uint_as_float(iz);
    const double r = z * invc - 1.0;
    const double y0 = logc + (double)k * LN2;
    const double r2 = r * r;
    double y = A1 * r + A2;
    y = A0 * r2 + y;
    y = y * r2 + (y0 + r);
    return (float)y;
}
__device__ __forceinline__ float log_filter(float v) /* filter_texture.h:62-67 */
{
    if ((double)v <= 1e-30)
        return 0.0f;
    return 0.5f + libm_logf(v) / 0.693147182f / 256.0f;
}
template <class T>
struct TLog /* LogTexture */
{
    __device__ static __forceinline__ V3 color(V3 p, const Env &e)
    {
        V3 c = T::color(p, e);
        return mk(log_filter(c.x), log_filter(c.y), log_filter(c.z));
    }
    __device__ static __forceinline__ float value(V3 p, const Env &e) { return mean3(color(p, e)); }
};
__device__ __forceinline__ V3 mirrorball_map(V3 v) /* transform_texture.h:46-59 */
{
    if (is_zero(v))
        return mk(0, 0, 0);
#if PT_FAST_MIRRORBALL /* cnormalize / csqrt / cdiv: the same bits as normalize, sqrtf and '/' */
    v = cnormalize(v);
#else
    v = PT_NORM(v);
#endif
    if (v.z <= -1.0f)
        return mk(0, 0.5f, 0);
#if PT_FAST_MIRRORBALL
    float d = csqrt(2.0f + 2.0f * v.z);
    if (d == 0.0f)
        return mk(0, 0.5f, 0);
    const Rcp rd = mkrcp(d);
    const bool dok = den_ok(d);
    float xt = cdiv(v.x, rd, dok), yt = cdiv(v.y, rd, dok);
#else
    float d = __builtin_sqrtf(2.0f + 2.0f * v.z);
    if (d == 0.0f)
        return mk(0, 0.5f, 0);
    float xt = v.x / d, yt = v.y / d;
#endif
    return mk((float)((double)xt * 0.5 + 0.5), (float)((double)yt * 0.5 + 0.5), 0);
}
/* The reference's std::atan2(float, float) and std::asin(float) are glibc's
 * atan2f / asinf (oracle.cpp SphericalTex), which are not correctly rounded
 * (16 % / 7 % of random operands differ from the rounded double result,
 * profiles/round3/glibc_atan2f_asinf_vs_double.txt).  Restated here: the
 * fdlibm float algorithms glibc 2.35 ships (flt-32 s_atanf / e_atan2f, and
 * e_asinf with its p0..p4 minimax), plain f32 arithmetic without contraction;
 * checked against glibc on the CPU (tools/libm: atan2f on 2e7 random
 * operands plus 2.4e6 edge operands -- exponent gaps of -140..127, signed
 * zeros, infinities, NaN --, asinf on every float in [-1, 1]: no
 * difference), and on the GPU against the host's glibc by pt_selftest_libm.
 *
 * fdlibm notice (the algorithms and constants below are Sun's):
 *   Copyright (C) 1993 by Sun Microsystems, Inc. All rights reserved.
 *   Developed at SunPro, a Sun Microsystems, Inc. business.
 *   Permission to use, copy, modify, and distribute this software is freely
 *   granted, provided that this notice is preserved.
 *   (Conversion to float by Ian Lance Taylor, Cygnus Support.) */
__device__ __forceinline__ float libm_atanf(float x)
{
    constexpr float hi[4] = {4.6364760399e-01f, 7.8539812565e-01f, 9.8279368877e-01f, 1.5707962513e+00f};
    constexpr float lo[4] = {5.0121582440e-09f, 3.7748947079e-08f, 3.4473217170e-08f, 7.5497894159e-08f};
    const int hx = __float_as_int(x), ix = hx & 0x7fffffff;
    int id;
    if (ix >= 0x4c000000) {
        if (ix > 0x7f800000)
            return x + x;
        return hx > 0 ? hi[3] + lo[3] : -hi[3] - lo[3];
    }
    if (ix < 0x3ee00000) {
        if (ix < 0x31000000)
            return x;
        id = -1;
    } else {
        x = __builtin_fabsf(x);
        if (ix < 0x3f980000) {
            if (ix < 0x3f300000)
                id = 0, x = (2.0f * x - 1.0f) / (2.0f + x);
            else
                id = 1, x = (x - 1.0f) / (x + 1.0f);
        } else {
            if (ix < 0x401c0000)
                id = 2, x = (x - 1.5f) / (1.0f + 1.5f * x);
            else
                id = 3, x = -1.0f / x;
        }
    }
    const float z = x * x, w = z * z;
    const float s1 = z * (3.3333334327e-01f + w * (1.4285714924e-01f + w * (9.0908870101e-02f +
                     w * (6.6610731184e-02f + w * (4.9768779427e-02f + w * 1.6285819933e-02f)))));
    const float s2 = w * (-2.0000000298e-01f + w * (-1.1111110449e-01f + w * (-7.6918758452e-02f +
                     w * (-5.8335702866e-02f + w * -3.6531571299e-02f))));
    if (id < 0)
        return x - x * (s1 + s2);
    const float r = (id == 0 ? hi[0] : id == 1 ? hi[1] : id == 2 ? hi[2] : hi[3]) -
                    ((x * (s1 + s2) - (id == 0 ? lo[0] : id == 1 ? lo[1] : id == 2 ? lo[2] : lo[3])) - x);
    return hx < 0 ? -r : r;
}
__device__ __forceinline__ float libm_atan2f(float y, float x)
{
    constexpr float PI_O_2 = 1.5707963705e+00f, PI_F = 3.1415927410e+00f, PI_LO = -8.7422776573e-08f;
    const int hx = __float_as_int(x), ix = hx & 0x7fffffff, hy = __float_as_int(y), iy = hy & 0x7fffffff;
    if (ix > 0x7f800000 || iy > 0x7f800000)
        return x + y;
    if (hx == 0x3f800000)
        return libm_atanf(y);
    int m = ((hy >> 31) & 1) | ((hx >> 30) & 2);
    if (iy == 0)
        return m == 0 || m == 1 ? y : m == 2 ? PI_F : -PI_F;
    if (ix == 0)
        return hy < 0 ? -PI_O_2 : PI_O_2;
    if (ix == 0x7f800000) {
        const float PI_O_4 = 7.8539818525e-01f;
        if (iy == 0x7f800000)
            return m == 0 ? PI_O_4 : m == 1 ? -PI_O_4 : m == 2 ? 3.0f * PI_O_4 : -3.0f * PI_O_4;
        return m == 0 ? 0.0f : m == 1 ? -0.0f : m == 2 ? PI_F : -PI_F;
    }
    if (iy == 0x7f800000)
        return hy < 0 ? -PI_O_2 : PI_O_2;
    const int k = (iy - ix) >> 23;
    float z;
    if (k > 60) /* glibc's flt-32 thresholds (FreeBSD's 26 with m &= 1 differs for gaps of 27..60) */
        z = PI_O_2 + 0.5f * PI_LO;
    else if (k < -60 && hx < 0)
        z = 0.0f;
    else
        z = libm_atanf(__builtin_fabsf(y / x));
    return m == 0 ? z : m == 1 ? -z : m == 2 ? PI_F - (z - PI_LO) : (z - PI_LO) - PI_F;
}
__device__ __forceinline__ float libm_asinf(float x)
{
    constexpr float PIO2_HI = 1.57079637050628662109375f, PIO2_LO = -4.37113900018624283e-8f,
                    PIO4_HI = 0.785398185253143310546875f;
    const int hx = __float_as_int(x), ix = hx & 0x7fffffff;
    auto poly = [](float t) {
        return t * (1.666675248e-1f + t * (7.495297643e-2f + t * (4.547037598e-2f + t * (2.417951451e-2f +
               t * 4.216630880e-2f))));
    };
    if (ix == 0x3f800000)
        return x * PIO2_HI + x * PIO2_LO;
    if (ix > 0x3f800000)
        return (x - x) / (x - x);
    if (ix < 0x3f000000) {
        if (ix < 0x32000000)
            return x;
        const float w = poly(x * x);
        return x + x * w;
    }
    float t = (1.0f - __builtin_fabsf(x)) * 0.5f;
    float p = poly(t);
    const float s = __builtin_sqrtf(t);
    if (ix >= 0x3F79999A) {
        t = PIO2_HI - (2.0f * (s + s * p) - PIO2_LO);
    } else {
        const float w = __int_as_float(__float_as_int(s) & 0xfffff000);
        const float c = (t - w * w) / (s + w);
        p = 2.0f * s * p - (PIO2_LO - 2.0f * c);
        t = PIO4_HI - (p - (PIO4_HI - 2.0f * w));
    }
    return hx > 0 ? t : -t;
}
__device__ __forceinline__ V3 spherical_map(V3 v) /* transform_texture.h:73-85 */
{
    const double PI = 3.14159265358979323846;
    if (is_zero(v))
        return mk(0, 0, 0);
    v = PT_NORM(v);
    float theta = libm_atan2f(v.y, v.x);
    if ((double)theta < -PI)
        theta = (float)((double)theta + 2 * PI);
    if ((double)theta > PI)
        theta = (float)((double)theta - 2 * PI);
    float phi = libm_asinf(v.z);
    return mk((float)((double)theta * 0.5 / PI + 0.5), (float)((double)phi / (PI / 2) * 0.5 + 0.5), 0);
}
template <class T>
struct TMirrorBall
{
    __device__ static __forceinline__ V3 color(V3 p, const Env &e) { return T::color(mirrorball_map(p), e); }
    __device__ static __forceinline__ float value(V3 p, const Env &e) { return T::value(mirrorball_map(p), e); }
};
template <class T>
struct TSpherical
{
    __device__ static __forceinline__ V3 color(V3 p, const Env &e) { return T::color(spherical_map(p), e); }
    __device__ static __forceinline__ float value(V3 p, const Env &e) { return T::value(spherical_map(p), e); }
};

/* Per-wave statistics, kept in LDS (every lane writes the same value). */
struct Counters
{
    u64 queries, leaf, attempts, rounds, shaded, nonleaf, slow, dark, mid;
#ifdef PT_PHASE_TIMING
    u64 ph[7]; /* cycles: generation, its attempts, fast pass, slow pass, accumulation, burst total, sample total */
    u64 ch[3]; /* cycles of the chunk loop: all of it, the lane-parallel front end, the result writes */
    u64 sp[3]; /* the spine's span queries: cycles, count, those that ran the lazy merge */
    u64 np[8]; /* events: bursts, loop iterations, (unused), fast passes, slow passes, accumulations, fast lanes, slow lanes */
#define PT_CNT(c, k, v) (c).np[k] += (v)
#else
#define PT_CNT(c, k, v)
#endif
};
/* ISA markers for static instruction counts (tools/isa_sections.py) */
#ifdef PT_MARKERS
#define PT_MARK(n) asm volatile("s_nop " #n)
#else
#define PT_MARK(n)
#endif
/* Per-phase wave cycle counters (profiling builds only: PT_DEVICE_DEFINES="PT_PHASE_TIMING") */
#ifdef PT_PHASE_TIMING
#define PT_T0(v) const u64 v = __builtin_amdgcn_s_memtime()
#define PT_ACC(c, k, v) (c).ph[k] += __builtin_amdgcn_s_memtime() - (v)
#define PT_ACC2(c, k, v) (c).ch[k] += __builtin_amdgcn_s_memtime() - (v)
#else
#define PT_ACC2(c, k, v)
#define PT_T0(v)
#define PT_ACC(c, k, v)
#endif

/* Statistics live in the wave's LDS Counters; lane 0 adds without a return
 * value (ds_add_u64), so no register carries them through the hot loops. */
__device__ __forceinline__ void cadd(u64 &c, u32 v)
{
    if ((threadIdx.x & 63) == 0)
        __hip_atomic_fetch_add(&c, (u64)v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
}

/* LCG jumps in LDS, shared by the workgroup's waves: j3[l] = (A, G * inc) of
 * 3l draws (attempt l of a round, lane l in attempt-major rounds; k < 8: the
 * offset of a lane-major round's k-th attempt), j24[l] = the same for
 * 3 PT_KATT l draws (lane l's first attempt, PT_KATT l, in a lane-major
 * round; 24l at the default 8).  Read where a
 * round needs them: hoisted out of the burst loop they would be held in
 * registers and spilled to scratch. */
struct JumpLds
{
    const u64 (*j3)[2];
    const u64 (*j24)[2];
};
__device__ __forceinline__ void jread(const u64 (*t)[2], int i, u64 &A, u64 &G)
{
    /* an index the compiler cannot see through: the load stays in the round
     * (a volatile load would lose the LDS address space and go through flat) */
    asm volatile("" : "+v"(i));
    A = t[i][0];
    G = t[i][1];
}
/* A burst-uniform struct parked in LDS, padded to whole 16-byte words so
 * that it is read with ds_read_b128 (a struct of floats is only 4-byte
 * aligned: the compiler would read it two words at a time). */
template <class T>
struct alignas(16) LdsBox
{
    static constexpr int N = (int)((sizeof(T) + 15) / 16);
    float4 w[N];
};
template <class T>
__device__ __forceinline__ T lds_get(const LdsBox<T> &b)
{
    union
    {
        float4 w[LdsBox<T>::N];
        T t;
    } u;
#pragma unroll
    for (int i = 0; i < LdsBox<T>::N; i++)
        u.w[i] = b.w[i];
    return u.t;
}
/* the same, each word kept a vector value (an empty asm on it): the
 * compiler cannot turn the uniform words into SGPRs, which a scene under
 * SGPR pressure spills into VGPR lanes and reads back one v_readlane at a time */
template <class T>
__device__ __forceinline__ T lds_get_v(const LdsBox<T> &b)
{
    union
    {
        float4 w[LdsBox<T>::N];
        T t;
    } u;
#pragma unroll
    for (int i = 0; i < LdsBox<T>::N; i++) {
        float4 v = b.w[i];
        asm volatile("" : "+v"(v.x), "+v"(v.y), "+v"(v.z), "+v"(v.w));
        u.w[i] = v;
    }
    return u.t;
}
template <class T>
__device__ __forceinline__ void lds_put(LdsBox<T> &b, const T &t)
{
    union
    {
        float4 w[LdsBox<T>::N];
        T t;
    } u;
    u.t = t;
#pragma unroll
    for (int i = 0; i < LdsBox<T>::N; i++)
        b.w[i] = u.w[i];
}
/* The wave index as a scalar (readfirstlane) or a vector value: a register
 * allocation choice with opposite effects per scene class (same-box A/B,
 * profiles/round4/ab_wave_index_ring_split.txt): Difference-free trees
 * (C2) +4.5 %, trees with a Difference (C3) -3.5 %, C5 +-0.  -1 = by scene. */
#ifndef PT_SCALAR_WAVE
#define PT_SCALAR_WAVE -1
#endif
/* the pass queries' primitive contexts as vector values (lds_get_v); same-box
 * A/B (profiles/round4/ab_ctx_vgpr.txt): C3 -0.8 %, C2 and C5 +-1 % -- off */
#ifndef PT_CTX_VGPR
#define PT_CTX_VGPR 0
#endif
/* the clear pass in union-only scenes too (round 2: off, C2 2.94 -> 3.37) */
#ifndef PT_CLEAR_UNION
#define PT_CLEAR_UNION 0
#endif
/* lane-major ring entries as two stores (C2 +8 %, C3 and C5 +-0, same A/B) */
/* lane index recomputed at each use in bursts (lane_id) or held in a
 * register; -1 = by scene: same-box A/B (profiles/round4/ab_lane_remat_lsum_lds.txt)
 * Difference-free trees (C2) +6 %, C3 -1 %, C5 -0.1 % */
#ifndef PT_LANE_REMAT
#define PT_LANE_REMAT -1
#endif
/* the fast order's lane sums in LDS instead of registers: -1 = where the
 * 768 B per wave leave the workgroups per CU unchanged (min_workgroups).
 * Off: C2 +1..2.5 % alone, nothing on top of PT_LANE_REMAT; C3, C5 +-0 */
#ifndef PT_LSUM_LDS
#define PT_LSUM_LDS 0
#endif
#ifndef PT_RING_SPLIT
#define PT_RING_SPLIT 1
#endif
#ifndef PT_LANE_MAJOR
#define PT_LANE_MAJOR 1 /* deferred rounds: lane l evaluates attempts 8l..8l+7 (one chained stream) */
#endif
#ifndef PT_LM_CHAINS
#define PT_LM_CHAINS 1 /* lane-major rounds: engine chains per lane (2: the halves interleaved) */
#endif
#ifndef PT_LM_BITS
#define PT_LM_BITS 1 /* lane-major rounds: per-lane bit planes + one wave prefix sum (burst_t) */
#endif
#ifndef PT_RING_FITS
#define PT_RING_FITS 1 /* PT_LM_BITS: the ring writes of a round whose kept attempts all fit skip the slot test */
#endif

#ifndef PT_PASS_PAIR_FALLBACK
/* 0: in a burst's fast pass over a Difference-free tree, lanes the one-pass
 * check cannot decide go to the full merge directly instead of through the
 * pairwise checks (whose all-pairs code raises the pass's register pressure
 * for lanes that are rare there) */
#define PT_PASS_PAIR_FALLBACK 0
#endif
/* Per-wave LDS work areas of the scatter loop. */
struct WaveLds
{
    void *ctx;            /* the burst origin's S::Root::Ctx, prepared once per burst     */
    float4 *ring;         /* PT_RCAP kept-child slots: parked ray, then the child's term */
    unsigned char *slowq; /* PT_SCAP slots waiting for the full merge (ring number mod 256) */
    unsigned char *midq;  /* PT_SCAP slots the clear pass could not finish (fast check next) */
    float *lsum;          /* the fast order's 64 lane sums, x / y / z planes (lsum_lds scenes) */
    float4 *stab;         /* PT_SPH_COMPACT: the burst origin's sphere contexts by primitive index */
    int *smat;            /* ... and their materials */
};

/* ---------------------------------------------------------------- spine --- */
/* One traceRay activation.  The current activation is F[sp]; all of its state
 * lives in LDS and is read where it is used, so the hot burst loop carries no
 * spine registers.  Every lane writes identical values. */
struct Frame
{
    V3 o, d;
    float strength;
    int depth;
    V3 hit, n;
    int mat;
    V3 retval;
    float add;
    V3 refl;
    float rf;
    V3 rc;
    float sc;
    V3 w; /* weight of the child being traced */
    int N, i, resume;
};

enum { B_DONE = 0, B_ABORT = 1, B_NONLEAF = 2 };

#ifndef PT_KATT
#define PT_KATT 8 /* rejection attempts per lane per generation round (A/B on C3: 4 -> 8 +6%) */
#endif
#ifndef PT_KATT_SHORT
/* per lane, in a short round; off (= PT_KATT) by default: short rounds of 2
 * cost C3 6 % (same-box A/B 143.4 vs 152.0 Msamples/s at 256 spp), and the
 * bursts they were for (matBrightDiffuseWhite's) are walked by lanes */
#define PT_KATT_SHORT PT_KATT
#endif
#ifndef PT_SHORT_REM
#define PT_SHORT_REM 24 /* children left at or below which a round is short (~91 attempts) */
#endif
#define PT_RCAP 256  /* kept-child slots per wave awaiting their lane-sum accumulation */
#define PT_SCAP 128  /* mid / slow queue entries (< 128 pending by construction; byte ring numbers) */
static_assert(PT_KATT % 2 == 0, "deferred rounds evaluate attempts in pairs");
#define PT_JUMP_ENTRIES 1025 /* host table: m = 0..1024 attempts */
static_assert(64 * PT_KATT < PT_JUMP_ENTRIES, "jump table too short for PT_KATT");
/* lane-major rounds count a lane's trailing failures in 4 balloted bit planes */
static_assert(PT_KATT <= 15, "a lane's trailing-failure count must fit 4 bits");
/* PT_LM_BITS: a round's totals in 10-bit fields of one packed wave prefix sum */
static_assert(64 * PT_KATT < 1024, "round totals must fit 10 bits");

/* One rejection attempt of the scatter loop body (path-trace.h:141-158):
 * s0 is the engine state before the attempt's three draws (outputs of s1, s2, s3). */
struct Attempt
{
    V3 wn;        /* accepted direction (unnormalised in deferred mode)      */
    float factor; /* 1 - (1 - dot(wn, n)) * sc (0 in deferred mode)         */
    u64 A, F, NL; /* wave ballots: accepted, hemisphere-failed, non-leaf    */
    bool acc;     /* this lane's attempt is accepted (its bit of A)         */
};

/* The predicates are balloted where they are produced, so they never pass
 * through a per-lane integer. */
template <bool DEFERRED, bool KR0>
__device__ __forceinline__ Attempt attempt(u64 s0, V3 n, V3 kR, float sc, float sNa, float abs_rc,
                                           bool child_leaf_depth)
{
    const W2 s1 = lcg_step({(u32)s0, (u32)(s0 >> 32)}), s2 = lcg_step(s1), s3 = lcg_step(s2);
    const V3 v = mk(u11(s1.hi), u11(s2.hi), u11(s3.hi));
    /* rand(): while (mag > max) with mag = sqrt(|v|^2); correctly rounded
     * sqrt(x) > 1  <=>  x > 1 + 2^-23 (exhaustively checked) */
    const bool ball = !(dot(v, v) > 0x1.000002p+0f);
    /* KR0: scatter coefficient 1 makes kR = 0 * reflectedRayDir = +-0 per
     * component, and v + +-0 == v because u11 never yields -0 */
    const V3 w = KR0 ? v : v + kR;
    const bool hemi = !(dot(n, w) <= EPS); /* while (dot(normal, dir) <= eps) */
    Attempt a;
    /* one ballot per compare (a ballot of a combined predicate is lowered
     * through a v_cndmask / v_cmp round trip) */
#ifdef PT_PAD_VALU /* experiment: extra independent VALU work per attempt */
    {
        float pad = v.x;
        for (int i = 0; i < PT_PAD_VALU; i++)
            asm volatile("v_add_f32 %0, %0, %0" : "+v"(pad));
        asm volatile("" ::"v"(pad));
    }
#endif
#ifdef PT_PAD_SALU /* experiment: extra SALU work per attempt */
    {
        int pad = 0;
        for (int i = 0; i < PT_PAD_SALU; i++)
            asm volatile("s_add_u32 %0, %0, 1" : "+s"(pad));
        asm volatile("" ::"s"(pad));
    }
#endif
    const u64 BB = __ballot(ball), HB = __ballot(hemi);
    a.A = BB & HB;
    a.F = BB & ~HB;
    a.acc = ball && hemi;
    a.wn = w;
    a.factor = 0.0f;
    a.NL = 0ull;
    if (!DEFERRED) {
        a.wn = cnormalize(w);
        a.factor = 1.0f - (1.0f - dot(a.wn, n)) * sc;
        const float cs = (sNa * a.factor) * abs_rc;
        a.NL = __ballot(ball && hemi && !(child_leaf_depth || cs < EPS));
    }
    return a;
}

/* Two attempts of a deferred burst (attempts k and k + 1 of a lane: engine
 * states s0a, s0b) in packed f32 (v_pk_fma / v_pk_mul / v_pk_add, one
 * instruction for both): element-wise the same IEEE operations in the same
 * order as attempt<true, KR0>, so the same bits. */
typedef float f2 __attribute__((ext_vector_type(2)));
struct Attempt2
{
    f2 x, y, z;   /* w of the two attempts (unnormalised)  */
    u64 A[2], F[2];
    bool acc[2];
};
template <bool KR0>
__device__ __forceinline__ Attempt2 attempt2_draws(W2 a1, W2 a2, W2 a3, W2 b1, W2 b2, W2 b3, V3 n, V3 kR);
template <bool KR0>
__device__ __forceinline__ Attempt2 attempt2(u64 s0a, u64 s0b, V3 n, V3 kR)
{
    const W2 a1 = lcg_step({(u32)s0a, (u32)(s0a >> 32)}), a2 = lcg_step(a1), a3 = lcg_step(a2);
    const W2 b1 = lcg_step({(u32)s0b, (u32)(s0b >> 32)}), b2 = lcg_step(b1), b3 = lcg_step(b2);
    return attempt2_draws<KR0>(a1, a2, a3, b1, b2, b3, n, kR);
}
/* Two CONSECUTIVE attempts of one lane's stream (lane-major rounds): the
 * second starts where the first's three draws end; s advances past both. */
template <bool KR0>
__device__ __forceinline__ Attempt2 attempt2_chain(u64 &s, V3 n, V3 kR)
{
    const W2 a1 = lcg_step({(u32)s, (u32)(s >> 32)}), a2 = lcg_step(a1), a3 = lcg_step(a2);
    const W2 b1 = lcg_step(a3), b2 = lcg_step(b1), b3 = lcg_step(b2);
    s = ((u64)b3.hi << 32) | (u64)b3.lo;
    return attempt2_draws<KR0>(a1, a2, a3, b1, b2, b3, n, kR);
}
/* Two attempts from two independent streams (sa, sb), each advanced past its
 * attempt's three draws: the two engine chains interleave. */
template <bool KR0>
__device__ __forceinline__ Attempt2 attempt2_split(u64 &sa, u64 &sb, V3 n, V3 kR)
{
    const W2 a1 = lcg_step({(u32)sa, (u32)(sa >> 32)}), b1 = lcg_step({(u32)sb, (u32)(sb >> 32)});
    const W2 a2 = lcg_step(a1), b2 = lcg_step(b1);
    const W2 a3 = lcg_step(a2), b3 = lcg_step(b2);
    sa = ((u64)a3.hi << 32) | (u64)a3.lo;
    sb = ((u64)b3.hi << 32) | (u64)b3.lo;
    return attempt2_draws<KR0>(a1, a2, a3, b1, b2, b3, n, kR);
}
template <bool KR0>
__device__ __forceinline__ Attempt2 attempt2_draws(W2 a1, W2 a2, W2 a3, W2 b1, W2 b2, W2 b3, V3 n, V3 kR)
{
    const f2 S = 0x1p-31f, M1 = -1.0f;
    /* u11: (float)o * 2^-31 - 1, the product exact (see u11) */
    f2 x = {(float)a1.hi, (float)b1.hi}, y = {(float)a2.hi, (float)b2.hi}, z = {(float)a3.hi, (float)b3.hi};
    x = __builtin_elementwise_fma(x, S, M1);
    y = __builtin_elementwise_fma(y, S, M1);
    z = __builtin_elementwise_fma(z, S, M1);
    const f2 vv = (x * x + y * y) + z * z; /* dot(v, v) */
    if (!KR0) {
        x = x + kR.x;
        y = y + kR.y;
        z = z + kR.z;
    }
#ifndef PT_HEMI_MODE
#define PT_HEMI_MODE 1 /* same-box A/B at 1024 spp on the round-6 kernel: 1 +0.9 % over 0 on C3, C2 +0.4..1.6 % (profiles/round6/ab_hemi_mode_r6.txt; round 5: 0 +0.9 % over 1; round 4: 1 +0.8 % over 0) */
#endif
#if PT_HEMI_MODE == 1
    /* dot(n, w) per attempt on scalar n (3 SGPRs rather than 3 splatted pairs) */
    const f2 nw = {(n.x * x.x + n.y * y.x) + n.z * z.x, (n.x * x.y + n.y * y.y) + n.z * z.y};
#elif PT_HEMI_MODE == 2
    /* the splatted normal in VGPRs (the asm hides its uniformity) */
    float vnx, vny, vnz;
    asm("v_mov_b32 %0, %1" : "=v"(vnx) : "s"(n.x));
    asm("v_mov_b32 %0, %1" : "=v"(vny) : "s"(n.y));
    asm("v_mov_b32 %0, %1" : "=v"(vnz) : "s"(n.z));
    const f2 nw = (x * vnx + y * vny) + z * vnz;
#else
    const f2 nw = (x * n.x + y * n.y) + z * n.z; /* dot(n, w): n.x * w.x == w.x * n.x */
#endif
    Attempt2 r;
    r.x = x, r.y = y, r.z = z;
    const bool ba = !(vv.x > 0x1.000002p+0f), bb = !(vv.y > 0x1.000002p+0f);
    const bool ha = !(nw.x <= EPS), hb = !(nw.y <= EPS);
    const u64 BA = __ballot(ba), HA = __ballot(ha), BBm = __ballot(bb), HBm = __ballot(hb);
    r.A[0] = BA & HA, r.F[0] = BA & ~HA, r.acc[0] = ba && ha;
    r.A[1] = BBm & HBm, r.F[1] = BBm & ~HBm, r.acc[1] = bb && hb;
    return r;
}

/* Replays the reference's sequential consumption of one half-round of 64
 * attempts (attempt j of the half = lane j) given its accept / hemisphere-
 * fail / non-leaf masks.  rem = children still to generate.  Returns the last
 * consumed attempt (63 when the whole half is consumed and no stop occurs);
 * sets `reason` on a stop and `take` = accepted leaf attempts consumed. */
__device__ __forceinline__ int replay(u64 A, u64 F, u64 NL, int rem, int &fails, int &reason, u64 &take)
{
    const int pa = __popcll(A), pf = __popcll(F);
    if (NL == 0ull && pa < rem && fails + pf < 1000) {
        /* common case: every attempt of the half is consumed */
        take = A;
        if (A) {
            const int last = 63 - __builtin_clzll(A);
            fails = (last == 63) ? 0 : __popcll(F >> (last + 1));
        } else {
            fails += pf;
        }
        return 63;
    }
    const int nl = NL ? __builtin_ctzll(NL) : 64;
    const int pos_rem = (pa >= rem) ? nth_set_bit(A, rem) : 64;
    int pos_abort = 64;
    if (fails + pf >= 1000) {
        int fc = fails;
        for (int l = 0; l < 64; l++) {
            if (l == nl || l == pos_rem)
                break;
            if ((A >> l) & 1ull)
                fc = 0;
            else if ((F >> l) & 1ull) {
                if (++fc == 1000) {
                    pos_abort = l;
                    break;
                }
            }
        }
    }
    if (pos_abort < 64 && pos_abort < nl && pos_abort < pos_rem) {
        reason = B_ABORT;
        take = A & ((1ull << pos_abort) - 1ull);
        return pos_abort;
    }
    if (nl < 64 && nl <= pos_rem) {
        reason = B_NONLEAF;
        take = A & ((1ull << nl) - 1ull);
        return nl;
    }
    if (pos_rem < 64) {
        reason = B_DONE;
        take = (pos_rem == 63) ? A : (A & ((2ull << pos_rem) - 1ull));
        return pos_rem;
    }
    take = A;
    if (A) {
        const int last = 63 - __builtin_clzll(A);
        fails = (last == 63) ? 0 : __popcll(F >> (last + 1));
    } else {
        fails += pf;
    }
    return 63;
}

/* Wave-cooperative scatter loop (path-trace.h:138-163) for sc > eps, from
 * child index f.i.  Each generation round evaluates 64*PT_KATT consecutive
 * rejection attempts, PT_KATT per lane (attempts l, 64 + l, ..: draws 3l..,
 * 192 + 3l.., ..),
 * replays the sequential rule on the ballots, and queues accepted leaf
 * children; every 64 queued children are traced one per lane.  Returns
 * B_DONE when all N children are summed, B_ABORT on the reference's
 * count > 1000 early return (path-trace.h:149-152), B_NONLEAF after writing
 * the next child's ray into `child` when that child must recurse (it draws
 * random numbers, so it runs on the spine). */
template <class S, bool STRICT, bool DEFERRED, bool KR0>
__device__ __forceinline__ int burst_t(const Env &e, Rng &rng, const u64 *__restrict__ jump, const JumpLds &J,
                                       const WaveLds &L, Frame &f, Frame &child, Counters &cnt)
{
    float4 *const ring = L.ring;
    unsigned char *const slowq = L.slowq, *const midq = L.midq;
    constexpr bool LANE_REMAT = PT_LANE_REMAT < 0 ? S::Root::NO_DIFF : PT_LANE_REMAT != 0;
    const int lane_reg = threadIdx.x & 63;
#define lane (LANE_REMAT ? lane_id() : lane_reg)
    const bool LSUM_LDS = L.lsum != nullptr; /* a constant: render_chunk sets it per scene */
    const V3 hit = univ(f.hit), n = univ(f.n), rc = univ(f.rc);
    const float sc = unif(f.sc), strength = unif(f.strength), add = unif(f.add);
    const int depth = uni(f.depth), N = uni(f.N);
    const int i = uni(f.i);
    V3 retval = univ(f.retval);
    const V3 kR = univ((1.0f / sc - 1.0f) * univ(f.refl)); /* (1 / scatter_coefficient - 1) * reflectedRayDir */
    const float sNa = unif((strength / (float)N) * add);  /* strength / scatter_ray_count * addFactor           */
    const float aN = unif(add / (float)N);                /* addFactor / scatter_ray_count                       */
    const float abs_rc = unif(length(rc));
    const bool child_leaf_depth = depth - 1 <= 0;
    /* lane l's state 3l draws into the round (attempt l): its jump (A, G)
     * is read from LDS where a round needs it, not held in registers */
    auto lane_state = [&]() {
        u64 jA, jG;
        jread(J.j3, lane, jA, jG);
        return jA * rng.st + jG;
    };
    /* lane-major rounds (deferred bursts): lane l's first attempt is 8l */
    constexpr bool LMAJ = DEFERRED && PT_LANE_MAJOR && PT_KATT_SHORT == PT_KATT;
    const u64 A64 = jump[128], g64inc = jump[129] * LCG_INC;   /* 64 attempts = 192 draws  */
    const u64 Afull = jump[128 * PT_KATT], gfullinc = jump[128 * PT_KATT + 1] * LCG_INC; /* a full round */
    int fails = 0, reason = -1;
    /* the burst origin's primitive contexts, shared by every pass of the burst
     * (and, in registers, by the generation rounds' dark test) */
    LdsBox<typename S::Root::Ctx> *const cxp = (LdsBox<typename S::Root::Ctx> *)L.ctx;
    typename S::Root::Ctx c0;
    S::Root::prep(c0, hit, e);
    lds_put(*cxp, c0);
    if constexpr (PT_SPH_COMPACT && Compact<typename S::Root>::OK)
        Compact<typename S::Root>::fill(L.stab, L.smat, c0);
    /* The burst's leaf children form one run of the fast order (oracle.cpp
     * ORDER_FAST): the run's non-zero terms are dealt round-robin to 64 lane
     * sums (lsum; the k-th one to lane k mod 64), which are added into retval
     * as their pairwise tree when the burst ends.  A DARK child (no emissive
     * primitive reachable, finite weight) has a zero term: the generation round
     * decides it on the accepted direction and it takes no memory at all.  Every
     * other child is KEPT: the round parks its direction in the slot ring
     * (numbered nkeep, in child order), where it waits for the passes, which
     * write its term back into the slot; slots are accumulated into the lane
     * sums in ring order once every slot before them is resolved.  npos counts
     * the burst's children.  In reference order (STRICT) every child is kept and
     * its term added to retval one by one (path-trace.h:160-162). */
    int npos = 0, nkeep = 0, keep_sum = 0, nzc = 0, f_n = 0, s_head = 0, s_n = 0, s_first = 0;
    int m_head = 0, m_n = 0, m_first = 0;
    V3 lsum = mk(0.0f, 0.0f, 0.0f);
    if (LSUM_LDS)
        L.lsum[lane] = L.lsum[64 + lane] = L.lsum[128 + lane] = 0.0f;
    int fast_on = 1, clear_on = 1;
    /* the clear pass applies when every emissive primitive hangs off the root
     * through Unions and transforms only */
    /* union-only scenes skip it: their first pass takes every primitive's
     * span and the union rule at once, which decides nearly every lane and
     * saves the mid queue's second pass (C2 2.94 -> 3.37 Msamples/s) */
    constexpr bool CLEAR = S::Root::template clear_ok<Emissive<S>>() && (PT_CLEAR_UNION || !S::Root::UNION_ONLY);
    /* RAW: dark children are decided on the unnormalised direction (dark_mask,
     * sound but conservative).  The zero term also needs a factor >= +0, i.e.
     * a computed dot(normalize(w), n) >= 0: accepted w have a computed
     * n.w > EPS and |w| <= 1 + |kR| (< 65), so the rounding of normalize and
     * dot (< 7e-5 here) cannot flip the sign.  Without RAW every child is kept
     * and the fast pass computes its exact term. */
    constexpr bool RAW = DEFERRED && !STRICT && S::Root::template raw_ok<Emissive<S>>();
    /* with the dark tests' burst-uniform preconditions folded in once per
     * burst: AND_p (ballot_p & pre_p) == (AND_p ballot_p) & AND_p pre_p.  A dark
     * child's term ((aN * factor) * rc) * (+0, +0, +0) is zero when the weight is
     * finite: aN <= 1, factor <= 1 + 2^-20, so |rc| < 1e37 per channel suffices
     * (NaN fails the compares: such bursts keep every child). */
    const bool wfin = __builtin_fabsf(rc.x) < 1e37f && __builtin_fabsf(rc.y) < 1e37f && __builtin_fabsf(rc.z) < 1e37f;
    const u64 raw_mask =
        uni_mask((KR0 || length(kR) < 64.0f) && wfin && S::Root::template dark_pre<Emissive<S>>(c0, e));
    /* children that enter a non-emissive plane before any emissive
     * primitive can be met are dark too (Occl, PT_OCCLUDE): occ_g = B 1.001 / T_E */
#if PT_OCCLUDE
    constexpr bool OCC = RAW && Occl<typename S::Root>::OK;
#else
    constexpr bool OCC = false;
#endif
    float occ_g = __builtin_inff();
    if constexpr (OCC) {
        const float te = fminf(Occl<typename S::Root>::template emis_lb<Emissive<S>>(c0, e), 1e19f);
        const float bw = (KR0 ? 1.0f : 1.0f + length(kR)) * 1.0001f;
        occ_g = unif(te > 0.0f ? bw * 1.001f / te : __builtin_inff());
    }
    auto dark = [&](V3 wn) -> u64 {
        u64 d = S::Root::template dark_mask<Emissive<S>>(c0, wn, e);
        if constexpr (OCC)
            d |= Occl<typename S::Root>::template occ<Emissive<S>>(c0, wn, occ_g, e);
        return d & raw_mask;
    };
    /* children recurse for factor >= eps / (sNa |rc|): short rounds when that
     * is below 0.99 (over 1 % of the children recurse) */
    const bool short_nd = !DEFERRED && EPS < 0.99f * (sNa * abs_rc);
    /* queued slots hold ring numbers mod 256; every pending one lies in
     * [keep_sum, keep_sum + PT_RCAP), which restores it */
    auto slot_pos = [&](unsigned char v) { return keep_sum + ((int)(v - keep_sum) & (PT_RCAP - 1)); };
    PT_CNT(cnt, 0, 1);
    for (;;) {
        PT_CNT(cnt, 1, 1);
        /* a round needs 64 free ring slots (more kept children than free slots
         * end the round early, below) */
        const bool room = PT_RCAP - (nkeep - keep_sum) >= 64;
        if (reason < 0 && room) {
            PT_T0(tg);
            PT_MARK(13);
            /* ---- generation round: lane l evaluates attempts l, 64 + l, ...
             * Each kept attempt's ring entry is written at once, as if
             * the whole round were consumed: a round that stops early consumes
             * a prefix of the accepted attempts, whose writes are the same, and
             * the rest lie past npos / nkeep, where nothing reads them before
             * a later round rewrites them.  Kept entries beyond the free ring
             * slots are not written (they could overwrite pending ones), and a
             * round consumes no kept child without a slot.  So the masks die
             * right after their writes, and only the rare round that stops
             * early needs them again: it evaluates the attempts a second time. */
            int rem = N - (i + npos);
            /* Short rounds (64 * PT_KATT_SHORT attempts) where a full round
             * would mostly be thrown away: a burst with few children left (a
             * recursing child's own small burst), or one whose children often
             * recurse -- a non-leaf child ends the round, and with factor =
             * 1 - (1 - cos) sc the child strength (sNa factor) |rc| reaches
             * eps for factor >= eps / (sNa |rc|) (matBrightDiffuseWhite's
             * bursts: a quarter of its children) */
            const int katt = (rem <= PT_SHORT_REM || (!DEFERRED && short_nd)) ? PT_KATT_SHORT : PT_KATT;
            int free_slots = PT_RCAP - (nkeep - keep_sum);
#ifdef PT_ROOM_CAP
            free_slots = min(free_slots, PT_ROOM_CAP); /* test hook: force early round ends */
#endif
            int ta = 0, tk = 0; /* accepted / kept attempts of the round */
            u64 nlor = 0ull, Alast = 0ull, Flast = 0ull;
            /* One attempt's ring entry (kept, with a free slot).  A deferred
             * burst parks the attempt's engine state (8 bytes, one register
             * pair): the first pass draws its three numbers again, which costs
             * less there -- 64 kept children per wave instruction -- than
             * moving the direction into a 16-byte store here, where a wave
             * instruction covers 64 attempts of which few are kept.  The
             * store runs under exec = kept mask & slot available. */
            const int slot_end = nkeep + free_slots;
            auto write_attempt = [&](u64 A, u64 kp, u64 st, V3 wn, float factor) {
                const int slot = mbcnt(kp, nkeep + tk);
                if (in_mask(kp & __ballot(slot < slot_end))) {
                    if (DEFERRED)
                        __builtin_memcpy(&ring[slot & (PT_RCAP - 1)], &st, 8);
                    else
                        ring[slot & (PT_RCAP - 1)] = make_float4(wn.x, wn.y, wn.z, factor);
                }
                ta += __popcll(A);
                tk += __popcll(kp);
            };
            int fails_lm = 0; /* lane-major: the consecutive failures after the round */
            if constexpr (LMAJ) {
                /* Lane-major round: lane l evaluates attempts 8l .. 8l+7, one
                 * chained stream (no jump between its attempts), in packed
                 * pairs.  Child order is attempt order j = 8l + k: the kept
                 * attempts of lanes below come first, so the ring slots are
                 * numbered once the round's kept masks are known, and a slot
                 * parks the lane's round state and k (the first pass jumps 3k
                 * draws).  tf = this lane's hemisphere failures after its
                 * last accepted attempt. */
                u64 jA, jG;
                jread(J.j24, lane, jA, jG);
                const u64 s_lane = jA * rng.st + jG;
#if PT_LM_BITS
                /* Per-lane bit planes, attempt k at bit KATT-1-k (one v_addc
                 * each: v + v + the balloted bit): accepted, hemisphere-failed
                 * and kept attempts.  The round's totals, each lane's count of
                 * kept attempts in the lanes below and the trailing failures
                 * then come from one wave prefix sum of the packed per-lane
                 * counts, and each lane writes its own kept attempts' ring
                 * entries in a loop over its set bits (as many trips as the
                 * most kept attempts of one lane) -- no per-attempt slot
                 * numbering or masked store block, and no kept-mask array in
                 * scalar registers. */
                u32 abits = 0u, fbits = 0u, kbits = 0u;
                u64 sk = s_lane;
#pragma unroll
                for (int k = 0; k < PT_KATT; k += 2) {
                    const Attempt2 ap = attempt2_chain<KR0>(sk, n, kR);
#pragma unroll
                    for (int h = 0; h < 2; h++) {
                        const V3 wn = h ? mk(ap.x.y, ap.y.y, ap.z.y) : mk(ap.x.x, ap.y.x, ap.z.x);
                        u64 D = 0ull;
                        if (RAW)
                            D = dark(wn);
                        abits = shl_lane_bit(abits, ap.A[h]);
                        fbits = shl_lane_bit(fbits, ap.F[h]);
                        kbits = shl_lane_bit(kbits, ap.A[h] & ~D);
                    }
                }
                /* failures after the lane's last accepted attempt (the bits
                 * below the lowest accepted one; none accepted: all of them) */
                const u32 tfl = (u32)__popc(fbits & ((abits & (0u - abits)) - 1u));
                /* packed per-lane counts: accepted | kept << 10 | trailing failures << 20
                 * (each total <= 64 KATT < 1024) */
                const u32 pk = (u32)__popc(abits) | ((u32)__popc(kbits) << 10) | (tfl << 20);
                const u32 incl = wave_incl_scan(pk), excl = incl - pk;
                const u32 tot = (u32)__builtin_amdgcn_readlane((int)incl, 63);
                ta = (int)(tot & 0x3FFu);
                tk = (int)((tot >> 10) & 0x3FFu);
                const u64 Aor = __ballot(abits != 0u);
                if (Aor) {
                    /* the trailing failures of lane L (the last with an accepted
                     * attempt) and of every lane above it */
                    const int L = 63 - __builtin_clzll(Aor);
                    fails_lm = (int)(tot >> 20) - (int)((u32)__builtin_amdgcn_readlane((int)excl, L) >> 20);
                } else {
                    fails_lm = fails + (int)(tot >> 20);
                }
                /* ring entries, numbered in child order: this lane's kept
                 * attempts follow those of the lanes below */
                int slot = nkeep + (int)((excl >> 10) & 0x3FFu);
                auto put = [&](u32 kb, bool check) {
                    for (; kb != 0u;) {
                        const int c = __builtin_clz(kb);
                        if (!check || slot < slot_end) {
                            float4 *r = &ring[slot & (PT_RCAP - 1)];
                            __builtin_memcpy(r, &s_lane, 8);
                            r->z = __int_as_float(c - (32 - PT_KATT)); /* attempt k of the lane */
                        }
                        slot++;
                        kb ^= 0x80000000u >> c;
                    }
                };
#if PT_RING_FITS
                /* the common round: every kept attempt has a free slot (a
                 * wave-uniform test once instead of a compare per entry) */
                if (tk <= free_slots)
                    put(kbits, false);
                else
#endif
                    put(kbits, true);
#else
                int tf = 0;
                u64 Aor = 0ull, K[PT_KATT];
#if PT_LM_CHAINS == 2
                /* two independent chains per lane: attempts k and k + KATT/2
                 * as one packed pair, the second chain starting 3 KATT/2
                 * draws into the lane's stream (one jump), so the pair's
                 * engine steps do not wait on each other; tfa / tfb = the
                 * trailing failures of each half, ab = the lane accepted in
                 * the second half */
                constexpr int HK = PT_KATT / 2;
                u64 sa = s_lane, sb;
                {
                    u64 hA, hG;
                    jread(J.j3, HK, hA, hG);
                    sb = hA * s_lane + hG;
                }
                int tfb = 0, ab = 0;
#pragma unroll
                for (int k = 0; k < HK; k++) {
                    const Attempt2 ap = attempt2_split<KR0>(sa, sb, n, kR);
#pragma unroll
                    for (int h = 0; h < 2; h++) {
                        const int kk = k + h * HK;
                        const V3 wn = h ? mk(ap.x.y, ap.y.y, ap.z.y) : mk(ap.x.x, ap.y.x, ap.z.x);
                        u64 D = 0ull;
                        if (RAW)
                            D = dark(wn);
                        K[kk] = ap.A[h] & ~D;
                        ta += __popcll(ap.A[h]);
                        tk += __popcll(K[kk]);
                        Aor |= ap.A[h];
                        if (h) {
                            tfb = zero_if(ap.A[h], add_lane_bit(tfb, ap.F[h]));
                            ab = mask_sel(ap.A[h], 1, ab);
                        } else {
                            tf = zero_if(ap.A[h], add_lane_bit(tf, ap.F[h]));
                        }
                    }
                }
                tf = ab ? tfb : tf + tfb;
#else
                u64 sk = s_lane;
#pragma unroll
                for (int k = 0; k < PT_KATT; k += 2) {
                    const Attempt2 ap = attempt2_chain<KR0>(sk, n, kR);
#pragma unroll
                    for (int h = 0; h < 2; h++) {
                        const V3 wn = h ? mk(ap.x.y, ap.y.y, ap.z.y) : mk(ap.x.x, ap.y.x, ap.z.x);
                        u64 D = 0ull;
                        if (RAW)
                            D = dark(wn);
                        K[k + h] = ap.A[h] & ~D;
                        ta += __popcll(ap.A[h]);
                        tk += __popcll(K[k + h]);
                        Aor |= ap.A[h];
                        tf = zero_if(ap.A[h], add_lane_bit(tf, ap.F[h]));
                    }
                }
#endif
                /* ring entries, numbered in child order */
                int slot = nkeep;
#pragma unroll
                for (int k = 0; k < PT_KATT; k++)
                    slot = mbcnt(K[k], slot);
#pragma unroll
                for (int k = 0; k < PT_KATT; k++) {
                    if (in_mask(K[k] & __ballot(slot < slot_end))) {
                        /* two stores, not one 16-byte one: a float4 of (state, k)
                         * would be one more 4-register value live across the loop */
#if PT_RING_SPLIT
                        float4 *r = &ring[slot & (PT_RCAP - 1)];
                        __builtin_memcpy(r, &s_lane, 8);
                        r->z = __int_as_float(k);
#else
                        ring[slot & (PT_RCAP - 1)] = make_float4(__uint_as_float((u32)s_lane),
                                                                 __uint_as_float((u32)(s_lane >> 32)),
                                                                 __int_as_float(k), 0.0f);
#endif
                    }
                    slot = add_lane_bit(slot, K[k]);
                }
                /* failures after the round's last accepted attempt (lane L,
                 * then every lane above it); none accepted: all of them */
                const u64 GE = Aor ? ~0ull << (63 - __builtin_clzll(Aor)) : ~0ull;
                int sf = 0;
#pragma unroll
                for (int b = 0; b < 4; b++)
                    sf += __popcll(__ballot((tf >> b) & 1) & GE) << b;
                fails_lm = Aor ? sf : fails + sf;
#endif
            } else if (DEFERRED) {
                /* pairs of attempts in packed f32 */
                u64 sk = lane_state();
#pragma unroll
                for (int k = 0; k < PT_KATT; k += 2) {
                    if (k >= katt)
                        break;
                    if (k)
                        sk = A64 * sk + g64inc;
                    const u64 sk1 = A64 * sk + g64inc;
                    const Attempt2 ap = attempt2<KR0>(sk, sk1, n, kR);
#pragma unroll
                    for (int h = 0; h < 2; h++) {
                        const V3 wn = h ? mk(ap.x.y, ap.y.y, ap.z.y) : mk(ap.x.x, ap.y.x, ap.z.x);
                        u64 D = 0ull;
                        if (RAW)
                            D = dark(wn);
                        write_attempt(ap.A[h], ap.A[h] & ~D, h ? sk1 : sk, wn, 0.0f);
                        if (k + h == katt - 1)
                            Alast = ap.A[h], Flast = ap.F[h];
                    }
                    sk = sk1;
                }
            } else {
                u64 sk = lane_state();
#pragma unroll
                for (int k = 0; k < PT_KATT; k++) {
                    if (k >= katt)
                        break;
                    if (k)
                        sk = A64 * sk + g64inc;
                    const Attempt at = attempt<DEFERRED, KR0>(sk, n, kR, sc, sNa, abs_rc, child_leaf_depth);
                    write_attempt(at.A, at.A, sk, at.wn, at.factor);
                    nlor |= at.NL;
                    if (k == katt - 1)
                        Alast = at.A, Flast = at.F;
                }
            }
            PT_ACC(cnt, 1, tg); /* the attempts alone (slot 1) */
#ifdef PT_FULL_STATS /* diagnostic builds: per-round attempt statistics */
            cadd(cnt.rounds, 1u);
#endif
            if (DEFERRED && KR0)
                PT_MARK(14); /* the diffuse (scatter coefficient 1) variant */
            int m; /* attempts consumed this round, 1..64*katt */
            int np, nk; /* children / kept children consumed */
            /* Common case: the whole round is consumed -- fewer accepted
             * children than remain, no non-leaf child, a slot for every kept
             * child, and no abort possible (fails + the round's 64 katt
             * attempts stay below 1000) -- so every half takes all its
             * accepted attempts, and the consecutive-failure count afterwards
             * is that of the last half, which has an accepted attempt. */
            if (nlor == 0ull && ta < rem && tk <= free_slots && fails <= 999 - 64 * katt && (LMAJ || Alast != 0ull)) {
                if (LMAJ) {
                    fails = fails_lm;
                } else {
                    const int last = 63 - __builtin_clzll(Alast);
                    fails = (last == 63) ? 0 : __popcll(Flast >> (last + 1));
                }
                m = 64 * katt;
                np = ta;
                nk = tk;
            } else {
                PT_COLD();
                /* ---- replay the sequential consumption rule half by half on
                 * the recomputed masks */
                Attempt at[PT_KATT];
                u64 Dm[PT_KATT];
                {
                    u64 sk = lane_state();
#pragma unroll
                    for (int k = 0; k < PT_KATT; k++) {
                        if (k)
                            sk = A64 * sk + g64inc;
                        at[k] = attempt<DEFERRED, KR0>(sk, n, kR, sc, sNa, abs_rc, child_leaf_depth);
                        Dm[k] = 0ull;
                        if (RAW)
                            Dm[k] = dark(at[k].wn);
                    }
                }
                m = 0;
                np = nk = 0;
                bool cut = false;
#pragma unroll
                for (int k = 0; k < PT_KATT; k++) {
                    if (reason < 0 && !cut && k < katt) {
                        u64 take = 0ull;
                        const int fails_in = fails;
                        const int c = replay(at[k].A, at[k].F, at[k].NL, rem, fails, reason, take);
                        m = 64 * k + c + 1;
                        rem -= __popcll(at[k].A);
                        u64 kp = take & ~Dm[k];
                        if (__popcll(kp) > free_slots) {
                            /* the slot ring is full: the round ends just before the
                             * first kept child without a slot (it is drawn again by
                             * the next round); no stop rule fired before it */
                            const int pos = nth_set_bit(kp, free_slots + 1);
                            const u64 pre = (1ull << pos) - 1ull;
                            take &= pre;
                            kp &= pre;
                            const u64 ca = at[k].A & pre;
                            if (ca) {
                                const int last = 63 - __builtin_clzll(ca);
                                fails = __popcll(at[k].F & pre & ~((2ull << last) - 1ull));
                            } else {
                                fails = fails_in + __popcll(at[k].F & pre);
                            }
                            reason = -1;
                            m = 64 * k + pos;
                            cut = true;
                        }
                        free_slots -= __popcll(kp);
                        np += __popcll(take);
                        nk += __popcll(kp);
                    }
                }
                if (!DEFERRED && reason == B_NONLEAF) {
                    const int l = (m - 1) & 63, kk = (m - 1) >> 6;
                    V3 wn = at[0].wn;
                    float fac = at[0].factor;
#pragma unroll
                    for (int k = 1; k < PT_KATT; k++)
                        if (kk == k)
                            wn = at[k].wn, fac = at[k].factor;
                    const V3 nd = mk(rdlane(wn.x, l), rdlane(wn.y, l), rdlane(wn.z, l));
                    const float nf = rdlane(fac, l);
                    /* w = addFactor / N * factor * reflect; strength = strength / N * addFactor * factor * |reflect| */
                    f.w = (aN * nf) * rc;
                    child.o = hit;
                    child.d = nd;
                    child.strength = (sNa * nf) * abs_rc;
                    child.depth = depth - 1;
                }
            }
#ifdef PT_FULL_STATS
            cadd(cnt.attempts, (u32)m);
#endif
            f_n += nk;
            npos += np;
            nkeep += nk;
            /* ---- advance the sample's stream past the consumed attempts */
            if (m == 64 * PT_KATT)
                rng.st = Afull * rng.st + gfullinc;
            else
                rng.st = jump[2 * m] * rng.st + jump[2 * m + 1] * LCG_INC;
            PT_ACC(cnt, 0, tg);
            PT_MARK(15);
        }
        const bool final = reason >= 0;
        /* drain everything when the next round would not fit */
        const bool drain = final || PT_RCAP - (nkeep - keep_sum) < 64;
        /* The fast check of one kept child (its normalised direction and
         * factor in en): true when its term is written to the ring, false
         * when it needs the full merge. */
        auto fast_lane = [&](int pos, float4 en) -> bool {
            const V3 dir = mk(en.x, en.y, en.z);
            PT_MARK(8);
#if PT_CTX_VGPR
            const typename S::Root::Ctx ctx = lds_get_v(*cxp);
#else
            const typename S::Root::Ctx ctx = lds_get(*cxp);
#endif
            int fok;
#if PT_UNION_FUSED && !PT_PASS_PAIR_FALLBACK
            if constexpr (PT_SPH_COMPACT && Compact<typename S::Root>::OK) {
                bool fh;
                float t;
                int mat;
                fok = compact_first_hit<typename S::Root>(ctx, mkray_unit(dir), e, L.stab, L.smat, fh, t, mat);
                if (fok) {
                    V3 col = mk(0, 0, 0);
                    if (fh)
                        col = S::emis(mat, hit + t * dir, e);
                    const V3 term = ((aN * en.w) * rc) * col;
                    ring[pos & (PT_RCAP - 1)] = make_float4(term.x, term.y, term.z, 0.0f);
                    return true;
                }
                return false;
            }
#endif
            PrimSpans<S::Root::HI> ps;
            PT_MARK(9);
            S::Root::span(ps, ctx, mkray_unit(dir), e);
            PT_MARK(10);
#if PT_UNION_FUSED && !PT_PASS_PAIR_FALLBACK
            if constexpr (S::Root::UNION_ONLY) {
                bool fh;
                float t;
                int mat;
                fok = union_first_hit<typename S::Root>(ps, fh, t, mat);
                PT_MARK(11);
                if (fok) {
                    V3 col = mk(0, 0, 0);
                    if (fh)
                        col = S::emis(mat, hit + t * dir, e);
                    PT_MARK(12);
                    const V3 term = ((aN * en.w) * rc) * col;
                    ring[pos & (PT_RCAP - 1)] = make_float4(term.x, term.y, term.z, 0.0f);
                    return true;
                }
                return false;
            }
#endif
            if constexpr (S::Root::NO_DIFF) {
                /* the union rule over the positive primitives (and empty
                 * intersections); the pairwise checks only where it cannot
                 * decide */
                fok = cheap_ok<typename S::Root>(ps);
#if PT_PASS_PAIR_FALLBACK
                if (wave_any(!fok)) {
                    if (!fok)
                        fok = S::Root::fast_ok(ps);
                }
#endif
            } else {
                fok = S::Root::fast_ok(ps);
            }
            PT_MARK(11);
            if (fok) {
                float t = 0.0f;
                int mat = 0;
                V3 col = mk(0, 0, 0);
                if (fast_first_hit<typename S::Root>(ps, t, mat))
                    col = S::emis(mat, hit + t * dir, e);
                PT_MARK(12);
                const V3 term = ((aN * en.w) * rc) * col;
                ring[pos & (PT_RCAP - 1)] = make_float4(term.x, term.y, term.z, 0.0f);
                return true;
            }
            return false;
        };
        /* Appends the lanes of SM (positions pos0 + lane, ring order) to a
         * queue of ring numbers. */
        auto enqueue = [&](unsigned char *q, int head, int &qn, int &qfirst, u64 SM, int pos0, int pos) {
            if ((SM >> lane) & 1ull)
                q[mbcnt(SM, head + qn) & (PT_SCAP - 1)] = (unsigned char)pos;
            if (qn == 0 && SM)
                qfirst = pos0 + __builtin_ctzll(SM);
            qn += __popcll(SM);
        };
        /* The passes below run as one scheduler: a queue is served as soon as
         * it holds 64 entries (partial batches only when draining and nothing
         * upstream is left), so the mid and slow queues never exceed 127
         * entries (PT_SCAP). */
        for (;;) {
            /* ---- stage C: slow passes, 64 parked children at a time through the
             * full merge */
            if (s_n > 0 && (s_n >= 64 || (drain && m_n == 0 && f_n == 0))) {
                PT_T0(tc);
                const int cs = s_n < 64 ? s_n : 64;
                PT_CNT(cnt, 4, 1);
                PT_CNT(cnt, 7, cs);
                if (lane < cs) {
                    const int pos = slot_pos(slowq[(s_head + lane) & (PT_SCAP - 1)]);
                    const float4 en = ring[pos & (PT_RCAP - 1)];
                    const V3 dir = mk(en.x, en.y, en.z);
                    const typename S::Root::Ctx ctx = lds_get(*cxp);
                    float t;
                    u32 ref;
                    bool ex;
                    V3 col = mk(0, 0, 0);
#ifndef PT_SLOW_STUB /* diagnostic builds only: the slow pass's merge left out (wrong bits) */
                    if (first_hit<typename S::Root>(ctx, dir, e, t, ref, ex))
                        col = S::emis(ref_mat(ref), hit + t * dir, e);
#else
                    (void)ctx, (void)t, (void)ref, (void)ex;
#endif
                    const V3 term = ((aN * en.w) * rc) * col;
                    ring[pos & (PT_RCAP - 1)] = make_float4(term.x, term.y, term.z, 0.0f);
                }
                s_head += cs;
                s_n -= cs;
                if (s_n)
                    s_first = slot_pos(uni(slowq[s_head & (PT_SCAP - 1)]));
                PT_ACC(cnt, 3, tc);
                continue;
            }
            /* ---- fast check on 64 children of the mid queue at a time (CLEAR
             * scenes); failing lanes go on to the full merge.  The mid queue is in
             * ring order, so the slow queue it feeds stays in ring order. */
            if (CLEAR && m_n > 0 && (m_n >= 64 || (drain && f_n == 0))) {
                PT_T0(tb);
                const int cm = m_n < 64 ? m_n : 64;
                int slow = 0, pos = 0;
                if (lane < cm) {
                    pos = slot_pos(midq[(m_head + lane) & (PT_SCAP - 1)]);
                    const float4 en = ring[pos & (PT_RCAP - 1)];
                    slow = (!fast_on || !fast_lane(pos, en)) ? 1 : 0;
                }
                const u64 SM = __ballot(slow);
                const int p0 = uni(__builtin_amdgcn_readlane(pos, SM ? __builtin_ctzll(SM) : 0));
                if ((SM >> lane) & 1ull)
                    slowq[mbcnt(SM, s_head + s_n) & (PT_SCAP - 1)] = (unsigned char)pos;
                if (s_n == 0 && SM)
                    s_first = p0;
                s_n += __popcll(SM);
                cadd(cnt.slow, (u32)__popcll(SM));
                if (fast_on && 4 * __popcll(SM) > 3 * cm)
                    fast_on = 0;
                m_head += cm;
                m_n -= cm;
                if (m_n)
                    m_first = slot_pos(uni(midq[m_head & (PT_SCAP - 1)]));
                PT_ACC(cnt, 2, tb);
                continue;
            }
            /* ---- first pass over the next 64 kept children (ring order).  With
             * CLEAR, lanes on which every non-emissive primitive is dead or ends
             * before EPS finish on the emissive primitives alone (about 4 in 5 of
             * C3's lit children); the others go to the mid queue for the fast
             * check.  Without CLEAR this is the fast check itself. */
            if (f_n > 0 && (f_n >= 64 || drain)) {
                PT_T0(tb);
                const int cf = f_n < 64 ? f_n : 64;
                const int pos0 = nkeep - f_n;
                const int pos = pos0 + lane;
                PT_CNT(cnt, 3, 1);
                PT_CNT(cnt, 6, cf);
                int park = 0; /* 1: mid queue, 2: slow queue */
                if (lane < cf) {
                    float4 en = ring[pos & (PT_RCAP - 1)];
                    if (DEFERRED) {
                        /* the parked attempt's three draws again (attempt2's
                         * arithmetic element by element: the same w), then the
                         * normalisation and factor of path-trace.h:157, :160,
                         * left to this pass so that 64 useful lanes do them */
                        u64 st;
                        __builtin_memcpy(&st, &en, 8);
                        if (LMAJ) { /* the lane's round state, then 3k draws to attempt k */
                            u64 jA, jG;
                            jread(J.j3, __float_as_int(en.z), jA, jG);
                            st = jA * st + jG;
                        }
                        const W2 s1 = lcg_step({(u32)st, (u32)(st >> 32)}), s2 = lcg_step(s1), s3 = lcg_step(s2);
                        V3 w = mk(u11(s1.hi), u11(s2.hi), u11(s3.hi));
                        if (!KR0)
                            w = w + kR;
                        const V3 nd = KR0 ? cnormalize_kept(w) : cnormalize(w);
                        /* KR0: sc == 1, and x * 1 == x */
                        en = make_float4(nd.x, nd.y, nd.z,
                                         KR0 ? 1.0f - (1.0f - dot(nd, n)) : 1.0f - (1.0f - dot(nd, n)) * sc);
                    }
                    if constexpr (CLEAR) {
                        park = 1;
                        if (clear_on) {
                            PT_MARK(16);
                            const V3 dir = mk(en.x, en.y, en.z);
                            const typename S::Root::Ctx ctx = lds_get(*cxp);
                            const Ray q = mkray_unit(dir);
                            const u64 CM = S::Root::template clear_mask<Emissive<S>, true>(ctx, q, e);
                            PrimSpans<S::Root::HI> ps;
                            S::Root::template span_sel<Emissive<S>>(ps, ctx, q, e);
                            if (((CM >> lane) & 1ull) && sel_ok<typename S::Root, Emissive<S>>(ps)) {
                                float t = 0.0f;
                                int mat = 0;
                                V3 col = mk(0, 0, 0);
                                if (sel_first_hit<typename S::Root, Emissive<S>>(ps, t, mat))
                                    col = S::emis(mat, hit + t * dir, e);
                                const V3 term = ((aN * en.w) * rc) * col;
                                ring[pos & (PT_RCAP - 1)] = make_float4(term.x, term.y, term.z, 0.0f);
                                park = 0;
                            }
                            PT_MARK(17);
                        }
                        if (DEFERRED && park)
                            ring[pos & (PT_RCAP - 1)] = en;
                    } else {
                        if (!fast_on || !fast_lane(pos, en)) {
                            /* park for the full merge */
                            park = 2;
                            if (DEFERRED)
                                ring[pos & (PT_RCAP - 1)] = en;
                        }
                    }
                }
                if constexpr (CLEAR) {
                    const u64 MM = __ballot(park == 1);
                    enqueue(midq, m_head, m_n, m_first, MM, pos0, pos);
                    cadd(cnt.mid, (u32)__popcll(MM));
                    /* the clear test keeps failing in this burst: stop trying */
                    if (clear_on && 4 * __popcll(MM) > 3 * cf)
                        clear_on = 0;
                } else {
                    const u64 SM = __ballot(park == 2);
                    enqueue(slowq, s_head, s_n, s_first, SM, pos0, pos);
                    cadd(cnt.slow, (u32)__popcll(SM));
                    /* overlap-heavy scenes (e.g. a box of sky half-spaces) stop trying */
                    if (fast_on && 4 * __popcll(SM) > 3 * cf)
                        fast_on = 0;
                }
                f_n -= cf;
                PT_ACC(cnt, 2, tb);
                continue;
            }
            break;
        }
        PT_T0(ts);
        /* ---- accumulate resolved slots in ring order: 64 at a time, fewer
         * only when draining.  Fast order: the batch's non-zero terms go to the
         * next lanes of the round-robin (lane (nzc + j) mod 64 for the batch's
         * j-th one) by one forward permute; the zero terms fill the remaining
         * lanes, where adding +-0 changes nothing (a lane sum starting at +0 is
         * never -0). */
        {
            int resolved = nkeep - f_n;
            if (m_n)
                resolved = min(resolved, m_first);
            if (s_n)
                resolved = min(resolved, s_first);
            while (resolved - keep_sum >= 64 || (drain && resolved > keep_sum)) {
                const int c = min(64, resolved - keep_sum);
                PT_CNT(cnt, 5, 1);
                V3 t = mk(0.0f, 0.0f, 0.0f);
                if (lane < c) {
                    const float4 tv = ring[(keep_sum + lane) & (PT_RCAP - 1)];
                    t = mk(tv.x, tv.y, tv.z);
                }
                if (STRICT) {
                    for (int j = 0; j < c; j++)
                        retval = retval + mk(rdlane(t.x, j), rdlane(t.y, j), rdlane(t.z, j));
                } else {
                    /* NaN compares unequal: a NaN term counts as non-zero, as in the oracle */
                    const u64 nz = __ballot(t.x != 0.0f) | __ballot(t.y != 0.0f) | __ballot(t.z != 0.0f);
                    const int pnz = __popcll(nz);
                    const int k = mask_sel(nz, mbcnt(nz, nzc), mbcnt(~nz, nzc + pnz));
                    const int to = (k & 63) << 2;
                    t = mk(__int_as_float(__builtin_amdgcn_ds_permute(to, __float_as_int(t.x))),
                           __int_as_float(__builtin_amdgcn_ds_permute(to, __float_as_int(t.y))),
                           __int_as_float(__builtin_amdgcn_ds_permute(to, __float_as_int(t.z))));
                    if (LSUM_LDS) {
                        float *const q = L.lsum;
                        const int l = lane;
                        q[l] = q[l] + t.x, q[64 + l] = q[64 + l] + t.y, q[128 + l] = q[128 + l] + t.z;
                    } else {
                        lsum = lsum + t;
                    }
                    nzc += pnz;
                }
                keep_sum += c;
            }
        }
        PT_ACC(cnt, 4, ts);
        if (final)
            break;
    }
    /* the run's end: retval + the pairwise tree of the 64 lane sums */
    if (!STRICT && npos > 0) {
        if (LSUM_LDS) {
            const int l = lane;
            lsum = mk(L.lsum[l], L.lsum[64 + l], L.lsum[128 + l]);
        }
        retval = wave_tree_sum3_add(lsum, retval);
    }
    /* leaf children of the burst (each one span query) and the dark ones among them */
    cadd(cnt.leaf, (u32)npos);
    cadd(cnt.dark, (u32)(npos - nkeep));
    f.retval = retval;
    f.i = i + npos;
    return reason;
}
#undef lane

/* Every child is provably a leaf when depth-1 <= 0 or when even the largest
 * possible factor (1 + 4e-7: wn and n are unit vectors) keeps the child
 * strength below eps.  Then acceptance needs no normalisation, and the
 * normalised direction / factor are computed per child at trace time (same
 * arithmetic, same bits) with every lane busy. */
template <class S, bool STRICT>
__device__ __forceinline__ int burst(const Env &e, Rng &rng, const u64 *__restrict__ jump, const JumpLds &jl,
                                     const WaveLds &L, Frame &f, Frame &child, Counters &cnt)
{
    const float sNa = unif((unif(f.strength) / (float)uni(f.N)) * unif(f.add));
    const float abs_rc = unif(length(univ(f.rc)));
    const bool deferred = uni(f.depth) - 1 <= 0 || (sNa * abs_rc * 1.01f < EPS);
    PT_T0(t0);
    int r;
    if (deferred) {
        if (unif(f.sc) == 1.0f)
            r = burst_t<S, STRICT, true, true>(e, rng, jump, jl, L, f, child, cnt);
        else
            r = burst_t<S, STRICT, true, false>(e, rng, jump, jl, L, f, child, cnt);
    } else {
        r = burst_t<S, STRICT, false, false>(e, rng, jump, jl, L, f, child, cnt);
    }
    PT_ACC(cnt, 5, t0);
    return r;
}

enum { PH_ENTER, PH_SETUP, PH_LOOP, PH_RETURN };
enum { RS_REFRACT, RS_SCATTER };

/* One sample = one traceRay tree (path-trace.h:58-165) + the jittered camera
 * ray of tracePixel (path-trace.h:190-198).  F = this wave's frame stack. */
/* A child of weight +-0 whose query need not run (PT_ZERO_CHILD).  The
 * reference folds a finished child as retval += w * r (path-trace.h:118,
 * :162).  A mirror child off a surface with reflectance 0 -- a sky or
 * emitter hit, which has no scatter loop -- has w = ((add / N) factor) rc =
 * +-0 and strength ... |rc| = 0 < eps, so its traceRay returns at once with
 * r = the emission where it lands, or 0 on a miss (path-trace.h:97-108).  When
 * every emission is finite (Scene::emis_finite: constant and image texels
 * bounded, codegen color_bound), w * r is +-0, and part + +-0 == part exactly
 * unless part is -0 or NaN -- checked here.  The skipped query still counts
 * as a query in the statistics. */
#ifndef PT_ZERO_CHILD
#define PT_ZERO_CHILD 1
#endif
__device__ __forceinline__ bool zero_child(V3 w, float cstr, int cdep, V3 part)
{
    const u32 wz = (__float_as_uint(w.x) | __float_as_uint(w.y) | __float_as_uint(w.z)) << 1;
    auto ok = [](float v) { return v == v && __float_as_uint(v) != 0x80000000u; };
    return wz == 0u && (cdep <= 0 || cstr < EPS) && ok(part.x) && ok(part.y) && ok(part.z);
}

/* The camera query of a sample, found ahead of time by one lane of the wave
 * (render_chunk traces a chunk's camera rays one per lane). */
struct CamHit
{
    int hit;
    float t;
    u32 ref;
    int ex;
};

/* tracePixel's jittered camera ray (path-trace.h:190-198): two draws */
__device__ __forceinline__ V3 camera_dir(const PtLaunch &lp, int pix, Rng &rng)
{
    const int px = pix % lp.gw, py = pix / lp.gw;
    float x = 2.0f * ((float)px + u01(rng_next(rng))) / (float)lp.W - 1.0f;
    float y = 1.0f - 2.0f * ((float)py + u01(rng_next(rng))) / (float)lp.H;
    return mk(x * lp.sw, y * lp.sh, -lp.dist);
}

/* A whole sample evaluated by one lane when its ray tree is the camera query
 * plus at most one mirror child that is a leaf (sky, background and other
 * non-scattering first hits).  Same statements as trace_sample's spine
 * (PH_ENTER / PH_SETUP / PH_LOOP / PH_RETURN) restricted to that shape;
 * returns false, leaving the sample to the wave, for any other shape.
 * nq / nsh = queries / shaded hits, for the statistics. */
template <class S>
__device__ __forceinline__ bool lane_sample(const Env &e, int depth, V3 o, V3 d, float strength, const CamHit &ch,
                                            V3 &res, int &nq, int &nsh)
{
    const V3 z = mk(0, 0, 0);
    nq = 1, nsh = 0;
    if (!ch.hit) {
        res = (z + mk(0, 0, 0)) / 1.0f;
        return true;
    }
    const V3 hit = o + ch.t * d;
    const int mat = ref_mat(ch.ref);
    V3 nn = S::Root::normal(ref_prim(ch.ref), ch.t, o, d, e);
    if (ch.ref & FLIP)
        nn = -nn;
    float ior;
    V3 n;
    if (ch.ex) {
        n = -nn;
        ior = S::ior(mat, e);
    } else {
        n = nn;
        ior = (float)(1.0 / (double)S::ior(mat, e));
    }
    const V3 retval = S::emis(mat, hit, e);
    const float add = 1.0f;
    if (depth <= 0 || strength < EPS) {
        res = (z + retval) / 1.0f;
        return true;
    }
    nsh = 1;
    const float rf = clamp01(S::trc(mat, hit, e)) * refract_strength(d, ior, n);
    if (rf > EPS)
        return false;
    const float sc = clamp01(S::scat(mat, hit, e));
    if (sc > EPS)
        return false;
    const float N = 1.0f; /* sc <= eps */
    const V3 rc = S::refl(mat, hit, e);
    const V3 refl = reflect(d, n);
    const float factor = 1.0f - (1.0f - dot(refl, n)) * sc;
    const V3 w = ((add / N) * factor) * rc;
    const float cs = (((strength / N) * add) * factor) * length(rc);
    if (!(depth - 1 <= 0 || cs < EPS))
        return false;
    nq = 2;
#if PT_ZERO_CHILD
    if constexpr (S::emis_finite)
        if (zero_child(w, cs, depth - 1, retval)) {
            res = (z + retval) / 1.0f;
            return true;
        }
#endif
    typename S::Root::Ctx ctx;
    S::Root::prep_l(ctx, hit, e);
    float t2 = 0.0f;
    u32 ref2 = 0;
    bool ex2 = false;
    V3 col = mk(0, 0, 0);
    if (lane_first_hit<typename S::Root>(ctx, refl, e, t2, ref2, ex2))
        col = S::emis(ref_mat(ref2), hit + t2 * refl, e);
    res = (z + (retval + w * col)) / 1.0f;
    return true;
}

#ifdef PT_LANE_WALK
/* A whole sample walked by its own lane when its ray tree has no scatter loop
 * (every node's scatter_coefficient <= eps: mirrors, glass, emitters --
 * C5's glass ball and sky box).  Such nodes draw no random numbers, so the
 * lanes of a chunk walk their trees independently: depth first, the
 * refraction child before the mirror child, each node the spine's own
 * statements (trace_sample PH_ENTER / PH_SETUP / PH_LOOP / PH_RETURN) and the
 * same fold retval = (e + w_R r_R) + w_M r_M.  Pending nodes live in a
 * PT_LANE_WALK-deep stack of register frames, shifted on push and pop (a
 * per-lane index would put it in scratch).  A lane whose tree needs a scatter
 * loop or a deeper stack gives the sample back to the wave (returns false).
 * nq / nsh = queries / shaded nodes, for the statistics. */
struct WalkFrame
{
    int mode;          /* 0: in R, M pending; 1: in R, no M; 2: in M */
    V3 part, wR, wM;   /* e (+ w_R r_R once R is done), the children's weights */
    V3 mo, md;         /* the M child's ray */
    float ms;          /* its strength */
    int mdep;          /* its depth */
};
template <class S, bool LIGHT = false>
__device__ __forceinline__ bool lane_walk(const Env &e, int depth0, V3 o0, V3 d0, float str0, const CamHit &ch,
                                          V3 &res, int &nq, int &nsh)
{
    constexpr int K = PT_LANE_WALK;
    WalkFrame F[K];
#pragma unroll
    for (int k = 0; k < K; k++)
        F[k].mode = 0;
    int sp = 0;
    V3 o = o0, d = d0, r = mk(0, 0, 0);
    int dep = depth0;
    float str = str0;
    bool first = true, descend = true, ok = true, done = false;
    nq = 0, nsh = 0;
    auto push = [&](const WalkFrame &w) {
#pragma unroll
        for (int k = K - 1; k > 0; k--)
            F[k] = F[k - 1];
        F[0] = w;
        sp++;
    };
    auto pop = [&]() {
#pragma unroll
        for (int k = 0; k < K - 1; k++)
            F[k] = F[k + 1];
        sp--;
    };
    while (ok && !done) {
        if (descend) {
            /* PH_ENTER */
            nq++;
            float t = 0.0f;
            u32 ref = 0;
            bool ex = false, found;
            if (first) {
                found = ch.hit != 0, t = ch.t, ref = ch.ref, ex = ch.ex != 0;
                first = false;
            } else {
                typename S::Root::Ctx ctx;
                S::Root::prep_l(ctx, o, e);
                if constexpr (LIGHT) {
                    /* a query the checks cannot decide: the full kernel's */
                    bool und;
                    found = lane_first_hit_light<typename S::Root>(ctx, d, e, t, ref, ex, und);
                    if (und) {
                        ok = false;
                        continue;
                    }
                } else {
                    found = lane_first_hit<typename S::Root>(ctx, d, e, t, ref, ex);
                }
            }
            if (!found) {
                r = mk(0, 0, 0);
                descend = false;
                continue;
            }
            const V3 hit = o + t * d;
            const int mat = ref_mat(ref);
            V3 nn = S::Root::normal(ref_prim(ref), t, o, d, e);
            if (ref & FLIP)
                nn = -nn;
            float ior;
            V3 n;
            if (ex) {
                n = -nn;
                ior = S::ior(mat, e);
            } else {
                n = nn;
                ior = (float)(1.0 / (double)S::ior(mat, e));
            }
            const V3 retval = S::emis(mat, hit, e);
            if (dep <= 0 || str < EPS) {
                r = retval;
                descend = false;
                continue;
            }
            nsh++;
            const float rf = clamp01(S::trc(mat, hit, e)) * refract_strength(d, ior, n);
            bool hasR = false;
            V3 rd = mk(0, 0, 0), wR = mk(0, 0, 0);
            float sR = 0.0f, add = 1.0f;
            if (rf > EPS) {
                rd = refract(d, ior, n);
                if (!is_zero(rd)) {
                    const V3 tr = S::trans(mat, hit, e);
                    wR = (1.0f * rf) * tr; /* addFactor * refractFactor * transmit */
                    sR = str * rf * 1.0f * length(tr);
                    hasR = true;
                    add = 1.0f * (1.0f - rf); /* PH_RETURN's addFactor *= 1 - rf */
                }
            }
            /* PH_SETUP */
            bool hasM = !(add < EPS);
            WalkFrame w;
            w.part = retval, w.wR = wR;
            w.wM = mk(0, 0, 0), w.mo = hit, w.md = mk(0, 0, 0), w.ms = 0.0f, w.mdep = dep - 1;
            if (hasM) {
                const float sc = clamp01(S::scat(mat, hit, e));
                if (sc > EPS) { /* a scatter loop: the wave's burst machinery */
                    ok = false;
                    continue;
                }
                /* N = 1 (sc <= eps) */
                const V3 rc = S::refl(mat, hit, e);
                const V3 refl = reflect(d, n);
                const float factor = 1.0f - (1.0f - dot(refl, n)) * sc;
                w.wM = ((add / 1.0f) * factor) * rc;
                w.md = refl;
                w.ms = (((str / 1.0f) * add) * factor) * length(rc);
            }
            /* a mirror child of weight +-0 (zero_child): without a refraction
             * child it is skipped here, with one once that child's sum is
             * known (mode 3) */
            bool zM = false;
#if PT_ZERO_CHILD
            if constexpr (S::emis_finite)
                zM = hasM && zero_child(w.wM, w.ms, w.mdep, hasR ? mk(0, 0, 0) : retval);
#endif
            if (zM && !hasR) {
                nq++;
                hasM = false;
            }
            if (!hasR && !hasM) {
                r = retval;
                descend = false;
                continue;
            }
            if (sp == K) { /* deeper than the register stack */
                ok = false;
                continue;
            }
            w.mode = hasR ? (hasM ? (zM ? 3 : 0) : 1) : 2;
            push(w);
            if (hasR)
                o = hit, d = rd, str = sR, dep = dep - 1;
            else
                o = w.mo, d = w.md, str = w.ms, dep = w.mdep;
        } else {
            /* PH_RETURN: fold the finished child into the top frame */
            if (sp == 0) {
                done = true;
                continue;
            }
            if (F[0].mode == 0 || F[0].mode == 3) {
                F[0].part = F[0].part + F[0].wR * r;
                if (F[0].mode == 3 && zero_child(F[0].wM, F[0].ms, F[0].mdep, F[0].part)) {
                    nq++; /* the mirror child's query, skipped */
                    r = F[0].part;
                    pop();
                    continue;
                }
                F[0].mode = 2;
                o = F[0].mo, d = F[0].md, str = F[0].ms, dep = F[0].mdep;
                descend = true;
            } else {
                r = F[0].part + (F[0].mode == 1 ? F[0].wR : F[0].wM) * r;
                pop();
            }
        }
    }
    if (!ok)
        return false;
    const V3 z = mk(0, 0, 0);
    res = (z + r) / 1.0f;
    return true;
}
#endif

#ifdef PT_LANE_SCATTER
/* A whole sample walked by its own lane, scatter loops included: the lane
 * draws its own engine's numbers in the reference's order (path-trace.h:
 * 138-163, one rejection attempt after another), so every recursing child's
 * subtree runs where it was generated, with no wave-level spine walk or burst
 * per child.  This is the shape of matBrightDiffuseWhite's samples (C2): ~10^4
 * children of which a quarter recurse, each into a dozen leaf children -- a
 * long chain of small loops that one wave would walk serially (~100 ms per
 * sample), while 64 lanes walk 64 such samples side by side.
 *
 * The fast order's run (oracle.cpp ORDER_FAST) is kept per lane for runs of at
 * most 64 non-zero terms: each lane sum then holds one term (+0 + t), and the
 * pairwise tree of the 64 lane sums is formed by a binary counter over the
 * terms in order, the empty lanes' +0 subtrees folded in at the flush.  A
 * 65th non-zero term, or a loop of more than 64 children likely to form one
 * run (a plain diffuse burst: the wave's machinery), gives the sample back to
 * the wave (returns false; the wave walks it again from its seed).  Pending
 * nodes live in a per-lane frame array (scratch): one push per recursing
 * child, the node being shaded stays in registers. */
struct ScFrame
{
    V3 hit, n, a, rc, part, w; /* a: incoming direction (refraction pending) or kR (loop) */
    float sc, str, add, rf;
    int dep, N, i, ms;         /* ms: material << 2 | stage */
};
enum { LS_AFTER_R = 0, LS_AFTER_M = 1, LS_LOOP = 2 };
#ifndef PT_LANE_RUN_CAP
#define PT_LANE_RUN_CAP 64 /* non-zero terms per run a lane keeps (test hook: fewer force hand-backs) */
#endif
static_assert(PT_LANE_RUN_CAP <= 64, "a lane's run holds at most one term per lane sum");
struct Run64
{
    V3 s[6], root;
    int m, len;
};
__device__ __forceinline__ void run_reset(Run64 &u) { u.m = 0, u.len = 0; }
/* adds one term; false on the 65th non-zero term */
__device__ __forceinline__ bool run_add(Run64 &u, V3 t)
{
    u.len++;
    if (t.x == 0.0f && t.y == 0.0f && t.z == 0.0f)
        return true;
    if (u.m == PT_LANE_RUN_CAP)
        return false;
    V3 v = mk(0.0f, 0.0f, 0.0f) + t; /* the lane sum: +0 + t */
    bool stored = false;
#pragma unroll
    for (int l = 0; l < 6; l++) {
        if (!stored) {
            if ((u.m >> l) & 1)
                v = u.s[l] + v;
            else
                u.s[l] = v, stored = true;
        }
    }
    if (!stored)
        u.root = v;
    u.m++;
    return true;
}
/* retval + the pairwise tree of the 64 lane sums (empty run: nothing) */
__device__ __forceinline__ V3 run_flush(Run64 &u, V3 retval)
{
    if (!u.len)
        return retval;
    V3 c = mk(0.0f, 0.0f, 0.0f);
    if (u.m == 64) {
        c = u.root;
    } else {
#pragma unroll
        for (int l = 0; l < 6; l++)
            c = ((u.m >> l) & 1) ? u.s[l] + c : c + mk(0.0f, 0.0f, 0.0f);
    }
    run_reset(u);
    return retval + c;
}

template <class S, int MAXD, bool STRICT>
__device__ __forceinline__ bool lane_walk_sc(const Env &e, int depth0, V3 o0, V3 d0, float str0, const CamHit &ch,
                                             Rng rng, V3 &res, int &nq, int &nsh)
{
    enum { ENTER, SETUP, LOOP, RETURN };
    ScFrame F[MAXD + 1];
    ScFrame c; /* the node being shaded */
    Run64 run;
    run_reset(run);
    int sp = 0, state = ENTER;
    V3 o = o0, d = d0, r = mk(0, 0, 0);
    int dep = depth0;
    float str = str0;
    bool first = true;
    nq = 0, nsh = 0;
    for (;;) {
        if (state == ENTER) {
            nq++;
            float t = 0.0f;
            u32 ref = 0;
            bool ex = false, found;
            if (first) {
                found = ch.hit != 0, t = ch.t, ref = ch.ref, ex = ch.ex != 0;
                first = false;
            } else {
                typename S::Root::Ctx ctx;
                S::Root::prep_l(ctx, o, e);
                found = lane_first_hit<typename S::Root>(ctx, d, e, t, ref, ex);
            }
            if (!found) {
                r = mk(0, 0, 0);
                state = RETURN;
                continue;
            }
            const V3 hit = o + t * d;
            const int mat = ref_mat(ref);
            V3 nn = S::Root::normal(ref_prim(ref), t, o, d, e);
            if (ref & FLIP)
                nn = -nn;
            float ior;
            V3 n;
            if (ex) {
                n = -nn;
                ior = S::ior(mat, e);
            } else {
                n = nn;
                ior = (float)(1.0 / (double)S::ior(mat, e));
            }
            const V3 retval = S::emis(mat, hit, e);
            if (dep <= 0 || str < EPS) {
                r = retval;
                state = RETURN;
                continue;
            }
            nsh++;
            c.hit = hit, c.n = n, c.a = d, c.part = retval, c.str = str, c.dep = dep, c.add = 1.0f;
            c.ms = mat << 2;
            const float rf = clamp01(S::trc(mat, hit, e)) * refract_strength(d, ior, n);
            c.rf = rf;
            state = SETUP;
            if (rf > EPS) {
                const V3 rd = refract(d, ior, n);
                if (!is_zero(rd)) {
                    const V3 tr = S::trans(mat, hit, e);
                    c.w = (1.0f * rf) * tr; /* addFactor * refractFactor * transmit */
                    c.ms |= LS_AFTER_R;
                    F[sp++] = c;
                    o = hit, d = rd, str = str * rf * 1.0f * length(tr), dep = dep - 1;
                    state = ENTER;
                }
            }
        } else if (state == SETUP) {
            if (c.add < EPS) {
                r = c.part;
                state = RETURN;
                continue;
            }
            const int mat = c.ms >> 2;
            const float sc = clamp01(S::scat(mat, c.hit, e));
            int N = cvt_x86(10000.0f * c.str * c.add * sc);
            if (sc <= EPS)
                N = 1;
            if (N == 0)
                N = 1;
            const V3 rc = S::refl(mat, c.hit, e);
            const V3 refl = reflect(c.a, c.n);
            if (!(sc > EPS)) { /* one mirror child, added on its own */
                const float Nf = (float)N;
                const float factor = 1.0f - (1.0f - dot(refl, c.n)) * sc;
                c.w = ((c.add / Nf) * factor) * rc;
                c.ms = (c.ms & ~3) | LS_AFTER_M;
                F[sp++] = c;
                o = c.hit, d = refl, str = (((c.str / Nf) * c.add) * factor) * length(rc), dep = c.dep - 1;
                state = ENTER;
                continue;
            }
            if (N > 64) {
                /* a loop likely to form a run of more than 64 terms: every
                 * child is a leaf, or few recurse (factor >= eps / (sNa |rc|)
                 * with factor = 1 - (1 - cos) sc) */
                const float sNa = (c.str / (float)N) * c.add, abs_rc = length(rc);
                const bool all_leaf = c.dep - 1 <= 0 || sNa * abs_rc * 1.01f < EPS;
                if (all_leaf || (1.0f - EPS / (sNa * abs_rc)) < 0.15f * sc)
                    return false;
            }
            c.a = (1.0f / sc - 1.0f) * refl; /* kR */
            c.sc = sc, c.rc = rc, c.N = N, c.i = 0;
            c.ms = (c.ms & ~3) | LS_LOOP;
            state = LOOP;
        } else if (state == LOOP) {
            if (c.i >= c.N) {
                r = run_flush(run, c.part);
                state = RETURN;
                continue;
            }
            const float sc = c.sc;
            const float sNa = (c.str / (float)c.N) * c.add, aN = c.add / (float)c.N, abs_rc = length(c.rc);
            /* path-trace.h:144-157: rand() redraws outside the unit ball, the
             * count > 1000 return after 1000 directions in the wrong hemisphere */
            V3 w;
            int fails = 0;
            bool abort = false;
            for (;;) {
                const float vx = u11(rng_next(rng)), vy = u11(rng_next(rng)), vz = u11(rng_next(rng));
                const V3 v = mk(vx, vy, vz);
                if (dot(v, v) > 0x1.000002p+0f)
                    continue;
                w = v + c.a;
                if (!(dot(c.n, w) <= EPS))
                    break;
                if (++fails == 1000) {
                    abort = true;
                    break;
                }
            }
            if (abort) {
                r = run_flush(run, c.part);
                state = RETURN;
                continue;
            }
            const V3 nd = cnormalize(w);
            const float factor = 1.0f - (1.0f - dot(nd, c.n)) * sc;
            const float cs = (sNa * factor) * abs_rc;
            if (c.dep - 1 <= 0 || cs < EPS) {
                /* a leaf child: its emission only */
                nq++;
                typename S::Root::Ctx ctx;
                S::Root::prep_l(ctx, c.hit, e);
                float t = 0.0f;
                u32 ref = 0;
                bool ex = false;
                V3 col = mk(0, 0, 0);
                if (lane_first_hit<typename S::Root>(ctx, nd, e, t, ref, ex))
                    col = S::emis(ref_mat(ref), c.hit + t * nd, e);
                const V3 term = ((aN * factor) * c.rc) * col;
                if (STRICT)
                    c.part = c.part + term;
                else if (!run_add(run, term))
                    return false;
                c.i++;
                continue;
            }
            /* a recursing child: the run so far closes, the child's subtree next */
            if (!STRICT)
                c.part = run_flush(run, c.part);
            c.w = (aN * factor) * c.rc;
            F[sp++] = c;
            o = c.hit, d = nd, str = cs, dep = c.dep - 1;
            state = ENTER;
        } else { /* RETURN */
            if (sp == 0)
                break;
            c = F[--sp];
            const int stage = c.ms & 3;
            if (stage == LS_AFTER_R) {
                c.part = c.part + c.w * r;
                c.add = 1.0f * (1.0f - c.rf);
                state = SETUP;
            } else if (stage == LS_AFTER_M) {
                r = c.part + c.w * r;
            } else {
                c.part = c.part + c.w * r;
                c.i++;
                state = LOOP;
            }
        }
    }
    const V3 z = mk(0, 0, 0);
    res = (z + r) / 1.0f;
    return true;
}
#endif

template <class S, int MAXD, bool STRICT>
__device__ __forceinline__ V3 trace_sample(const Env &e, const PtLaunch &lp, int pix, int s, Frame *F, const WaveLds &L,
                                           const u64 *__restrict__ jump, const JumpLds &jl, Counters &cnt,
                                           const CamHit &cam)
{
    Rng rng;
    rng_seed(rng, lp.seed, PT_ITEM_KEY(lp, pix), (u64)s);
#ifdef PT_RAYS
    /* traceRay(ray, it, depth, engine, strength): the caller's ray, no camera draws */
    {
        const float *r = lp.rays + 7 * (long long)pix;
        F[0].o = mk(r[0], r[1], r[2]);
        F[0].d = mk(r[3], r[4], r[5]);
        F[0].strength = r[6];
    }
#else
    F[0].o = mk(0, 0, 0);
    F[0].d = camera_dir(lp, pix, rng);
    F[0].strength = 1.0f;
#endif
    F[0].depth = lp.depth;
    int sp = 0;
    int phase = PH_ENTER;
    V3 result = mk(0, 0, 0);
    for (;;) {
        Frame &f = F[sp];
        if (phase == PH_ENTER) {
            cnt.queries++;
            const V3 o = univ(f.o), d = univ(f.d);
            float t = 0.0f;
            u32 ref = 0;
            bool ex = false;
            bool found;
            if (sp == 0) {
                found = cam.hit != 0, t = cam.t, ref = cam.ref, ex = cam.ex != 0;
            } else {
                PT_T0(tq);
                typename S::Root::Ctx ctx;
                S::Root::prep(ctx, o, e);
#ifdef PT_FAST_SPINE /* per scene, pt_scene_set_fast_spine */
                int merged = 0;
                found = spine_first_hit<typename S::Root>(ctx, d, e, t, ref, ex, merged);
#ifdef PT_PHASE_TIMING
                cnt.sp[2] += (u64)merged;
#endif
#else
                found = first_hit<typename S::Root>(ctx, d, e, t, ref, ex);
#endif
#ifdef PT_PHASE_TIMING
                cnt.sp[0] += __builtin_amdgcn_s_memtime() - tq;
                cnt.sp[1]++;
#endif
            }
            if (!found) {
                result = mk(0, 0, 0);
                phase = PH_RETURN;
                continue;
            }
            t = unif(t);
            ref = (u32)uni((int)ref);
            const V3 hit = o + t * d;
            const int mat = ref_mat(ref);
            V3 nn = S::Root::normal(ref_prim(ref), t, o, d, e);
            if (ref & FLIP)
                nn = -nn;
            float ior;
            V3 n;
            if (ex) {
                n = -nn;
                ior = S::ior(mat, e);
            } else {
                n = nn;
                ior = (float)(1.0 / (double)S::ior(mat, e));
            }
            const V3 retval = S::emis(mat, hit, e);
            f.hit = hit, f.n = n, f.mat = mat, f.retval = retval, f.add = 1.0f;
            const float strength = unif(f.strength);
            if (uni(f.depth) <= 0 || strength < EPS) {
                result = retval;
                phase = PH_RETURN;
                continue;
            }
            cnt.shaded++;
            const float rf = clamp01(S::trc(mat, hit, e)) * refract_strength(d, ior, n);
            f.rf = rf;
            if (rf > EPS) {
                V3 rd = refract(d, ior, n);
                if (!is_zero(rd)) {
                    V3 tr = S::trans(mat, hit, e);
                    f.w = (1.0f * rf) * tr; /* addFactor * refractFactor * transmit, addFactor == 1 */
                    f.resume = RS_REFRACT;
                    Frame &c = F[sp + 1];
                    c.o = hit, c.d = rd;
                    c.strength = strength * rf * 1.0f * length(tr);
                    c.depth = uni(f.depth) - 1;
                    sp++;
                    continue;
                }
            }
            phase = PH_SETUP;
        } else if (phase == PH_SETUP) {
            const float add = unif(f.add);
            if (add < EPS) {
                result = univ(f.retval);
                phase = PH_RETURN;
                continue;
            }
            const int mat = uni(f.mat);
            const V3 hit = univ(f.hit), n = univ(f.n);
            const float sc = clamp01(S::scat(mat, hit, e));
            int N = cvt_x86(10000.0f * unif(f.strength) * add * sc);
            if (sc <= EPS)
                N = 1;
            if (N == 0)
                N = 1;
            f.sc = sc, f.N = N, f.i = 0;
            f.rc = S::refl(mat, hit, e);
            f.refl = reflect(univ(f.d), n);
            phase = PH_LOOP;
        } else if (phase == PH_LOOP) {
            if (uni(f.i) >= uni(f.N)) {
                result = univ(f.retval);
                phase = PH_RETURN;
                continue;
            }
            if (unif(f.sc) > EPS) {
                int why = burst<S, STRICT>(e, rng, jump, jl, L, f, F[sp + 1], cnt);
                if (why != B_NONLEAF) {
                    result = univ(f.retval);
                    phase = PH_RETURN;
                    continue;
                }
                cnt.nonleaf++;
                f.resume = RS_SCATTER;
                sp++;
                phase = PH_ENTER;
            } else {
                const V3 refl = univ(f.refl), n = univ(f.n), rc = univ(f.rc);
                const float sc = unif(f.sc), add = unif(f.add), N = (float)uni(f.N);
                float factor = 1.0f - (1.0f - dot(refl, n)) * sc;
                const V3 w = ((add / N) * factor) * rc;
                const float cstr = (((unif(f.strength) / N) * add) * factor) * length(rc);
#if PT_ZERO_CHILD
                if constexpr (S::emis_finite)
                    if (zero_child(w, cstr, uni(f.depth) - 1, univ(f.retval))) {
                        cnt.queries++; /* the child's query, skipped */
                        f.i = uni(f.i) + 1;
                        continue;
                    }
#endif
                f.w = w;
                f.resume = RS_SCATTER;
                Frame &c = F[sp + 1];
                c.o = univ(f.hit), c.d = refl;
                c.strength = cstr;
                c.depth = uni(f.depth) - 1;
                sp++;
                phase = PH_ENTER;
            }
        } else { /* PH_RETURN */
            if (sp == 0)
                break;
            sp--;
            Frame &p = F[sp];
            p.retval = univ(p.retval) + univ(p.w) * result;
            if (uni(p.resume) == RS_REFRACT) {
                p.add = unif(p.add) * (1.0f - unif(p.rf));
                phase = PH_SETUP;
            } else {
                p.i = uni(p.i) + 1;
                phase = PH_LOOP;
            }
        }
    }
    /* tracePixel with one sample: (Color(0,0,0) + traceRay(...)) / 1 */
    V3 z = mk(0, 0, 0);
    return (z + result) / 1.0f;
}

#ifndef PT_WPW
#define PT_WPW 4 /* independent waves per workgroup */
#endif
/* Work item -> (pixel slot, sample).  Sample-major (small launches, chosen
 * by the runtime): consecutive items are consecutive slots at one sample, so
 * a dequeued chunk holds one sample of each of CH neighbouring pixels and an
 * expensive pixel's samples spread over many chunks -- slot-major chunks
 * hold up to CH samples of one pixel, and one wave could draw hundreds of ms
 * of work near the end of a launch (C3 at 16 spp: 73 Msamples/s slot-major,
 * 98 sample-major).  Large launches stay slot-major: their last chunks are
 * the frame's last pixels, a short tail (C3 at 128 spp: sample-major -2 %).
 * Results do not depend on the order: every (pixel, sample) is seeded by its
 * own indices and the stage buffer is indexed slot-major either way. */
__device__ __forceinline__ void item_slot(const PtLaunch &lp, long long item, long long &slot, int &s)
{
    if (lp.sample_major) {
        const long long nslots = lp.n_items / lp.nsamp;
        const long long k = item / nslots;
        slot = item - k * nslots;
        /* a chunk's slots spread over the pixel list: the expensive pixels of
         * a small launch (a mirror's reflection, clustered in the list) do not
         * fall into one wave's chunk, which it would walk one by one */
        if (lp.perm)
            slot = (long long)(((unsigned long long)slot * (unsigned long long)lp.perm) % (unsigned long long)nslots);
        s = lp.s0 + (int)k;
    } else {
        slot = item / lp.nsamp;
        s = lp.s0 + (int)(item - slot * lp.nsamp);
    }
}
#ifndef PT_CHUNK
#define PT_CHUNK 64 /* default (pixel, sample) items a wave takes per dequeue (<= 64) */
#endif
/* the next chunk's dequeue issued before this chunk's work (the atomic's wait
 * joins the chunk's first load).  Same-box A/B, round 4
 * (profiles/round4/ab_knobs_r4u.txt): C3 -0.5 %, C5 (lane walks) +0.36 %:
 * on for lane-walk scenes */
/* the run-taking work queue, compiled where the runtime asks for runs
 * (lane-walk scenes); other scenes keep one chunk per atomic */
#ifndef PT_GRAB_RUNS
#if defined(PT_LANE_WALK) || defined(PT_LANE_SCATTER)
#define PT_GRAB_RUNS 1
#else
#define PT_GRAB_RUNS 0
#endif
#endif
#ifndef PT_GRAB_TICKS
#define PT_GRAB_TICKS 20000 /* 200 us per chunk at the 100 MHz real-time clock */
#endif
#ifndef PT_DEQUEUE_PREFETCH
#if defined(PT_LANE_WALK)
#define PT_DEQUEUE_PREFETCH 1
#else
#define PT_DEQUEUE_PREFETCH 0
#endif
#endif

/* Workgroups per CU for the launch bounds: 5 (5 waves/SIMD, VGPRs capped at
 * 96; A/B on C3: 4 -> 5 +6.6 %, 3 -> -13 %) when that many workgroups' LDS
 * fits the CU's 160 KB, else as many as fit -- the frame stack grows with
 * MAXD (depth 16: 4, depth 64: 2), and a cap whose extra wave cannot be
 * resident would only spill registers. */
template <class S, int MAXD, bool LSUM>
__device__ constexpr int lds_workgroups()
{
    constexpr int lds = PT_WPW * ((MAXD + 1) * (int)sizeof(Frame) + 16 * PT_RCAP + 2 * PT_SCAP +
                                  (int)sizeof(Counters) + (int)sizeof(LdsBox<typename S::Root::Ctx>) + 64 * 16 +
                                  (LSUM ? 3 * 64 * 4 : 4)) +
                        2 * 64 * 16;
    constexpr int alloc = (lds + 1279) / 1280 * 1280; /* gfx950 LDS allocation unit (measured) */
    constexpr int n = 160 * 1024 / alloc;
    return n < 1 ? 1 : n > 5 ? 5 : n;
}
/* lane sums in LDS (PT_LSUM_LDS): forced, or where they cost no workgroup per CU */
template <class S, int MAXD>
__device__ constexpr bool lsum_lds()
{
    return PT_LSUM_LDS < 0 ? lds_workgroups<S, MAXD, true>() == lds_workgroups<S, MAXD, false>() : PT_LSUM_LDS != 0;
}
template <class S, int MAXD>
__device__ constexpr int min_workgroups()
{
    return lds_workgroups<S, MAXD, lsum_lds<S, MAXD>()>();
}

/* The megakernel body.  Persistent: the grid is sized to the resident
 * capacity and every wave pulls 64-item chunks from a global counter until
 * none are left.  Per-chunk cost varies by ~10^5 (sky pixels vs diffuse
 * pixels), so static assignment or one-chunk-per-wave launches leave most
 * SIMDs idle behind the slowest wave of each workgroup. */
template <class S, int MAXD, bool STRICT, bool LIGHT = false>
__device__ __forceinline__ void render_chunk(const float *__restrict__ P, const PtImage *__restrict__ imgs,
                                             const u64 *__restrict__ jump, float *__restrict__ out,
                                             const int *__restrict__ pixels, u64 *__restrict__ stats,
                                             const PtLaunch &lp)
{
    __shared__ Frame stk[PT_WPW][MAXD + 1];
    __shared__ LdsBox<typename S::Root::Ctx> xbuf[PT_WPW];
    __shared__ float4 rbuf[PT_WPW][PT_RCAP];
    __shared__ unsigned char sbuf[PT_WPW][PT_SCAP];
    __shared__ unsigned char mbuf[PT_WPW][PT_SCAP];
    __shared__ Counters cbuf[PT_WPW];
    constexpr bool LSUM_LDS = lsum_lds<S, MAXD>();
    __shared__ float lsbuf[PT_WPW][LSUM_LDS ? 3 * 64 : 1];
    constexpr bool SCOMPACT = PT_SPH_COMPACT && Compact<typename S::Root>::OK;
    __shared__ float4 stbuf[PT_WPW][SCOMPACT ? S::Root::HI : 1];
    __shared__ int smbuf[PT_WPW][SCOMPACT ? S::Root::HI : 1];
    /* a chunk's lanes while the wave walks its samples one by one: (pixel,
     * sample | hit << 30 | exit << 31, camera t, camera ref), replaced by the
     * sample's result (x, y, z) once it is traced; in LDS rather than in
     * registers that would stay live through every burst (the allocator
     * spilled them to scratch) */
    __shared__ uint4 lbuf[PT_WPW][64];
    /* engine jumps of 3l and 24l draws (A, G * inc): JumpLds */
    __shared__ u64 jbuf[64][2];
    __shared__ u64 jbuf24[64][2];
    constexpr bool SCALAR_WAVE = PT_SCALAR_WAVE < 0 ? S::Root::NO_DIFF : PT_SCALAR_WAVE != 0;
    const int wave = SCALAR_WAVE ? __builtin_amdgcn_readfirstlane(threadIdx.x >> 6) : threadIdx.x >> 6;
    const int lane = threadIdx.x & 63;
    const u64 t_start = __builtin_amdgcn_s_memrealtime(); /* 100 MHz: wave lifetimes, stats[26..29] */
    const Env e = {P, imgs};
#ifdef PT_POISON_LDS
    /* test build: every LDS word starts as all-ones (NaN floats, ring numbers
     * 255, -1 integers) instead of whatever the CU's previous workgroup left,
     * so a read of LDS state this launch has not written changes the bits
     * (round 2's kept-only position flags read stale flags in small launches) */
    {
        auto poison = [&](void *p, unsigned bytes) {
            for (unsigned k = threadIdx.x; k < bytes / 4; k += blockDim.x)
                ((u32 *)p)[k] = 0xFFFFFFFFu;
        };
        poison(stk, sizeof stk), poison(xbuf, sizeof xbuf), poison(rbuf, sizeof rbuf), poison(sbuf, sizeof sbuf);
        poison(mbuf, sizeof mbuf), poison(cbuf, sizeof cbuf), poison(lbuf, sizeof lbuf);
        poison(jbuf, sizeof jbuf), poison(jbuf24, sizeof jbuf24);
        __syncthreads();
    }
#endif
    for (int i = threadIdx.x; i < 128; i += 64 * PT_WPW) {
        const int l = i & 63, m = i < 64 ? l : PT_KATT * l; /* m attempts = 3m draws */
        u64 *t = i < 64 ? jbuf[l] : jbuf24[l];
        t[0] = jump[2 * m], t[1] = jump[2 * m + 1] * LCG_INC;
    }
    __syncthreads();
    const JumpLds jl = {jbuf, jbuf24};
    Counters &cnt = cbuf[wave];
    cnt.queries = cnt.leaf = cnt.attempts = cnt.rounds = cnt.shaded = cnt.nonleaf = cnt.slow = cnt.dark = 0;
    cnt.mid = 0;
#ifdef PT_PHASE_TIMING
    for (int k = 0; k < 7; k++)
        cnt.ph[k] = 0;
    for (int k = 0; k < 8; k++)
        cnt.np[k] = 0;
    cnt.sp[0] = cnt.sp[1] = cnt.sp[2] = 0;
    cnt.ch[0] = cnt.ch[1] = cnt.ch[2] = 0;
#endif
    const WaveLds L = {&xbuf[wave], rbuf[wave], sbuf[wave], mbuf[wave], LSUM_LDS ? lsbuf[wave] : nullptr,
                       stbuf[wave], smbuf[wave]};
    const int CH = lp.chunk > 0 ? lp.chunk : PT_CHUNK; /* small launches use smaller chunks */
    const long long n_chunks = (lp.n_items + CH - 1) / CH;
    /* Split launches (lane-walk scenes, see pt_render_light): the full kernel
     * serves the light kernel's list, with its own counter (stats[36]) */
    u64 *work = stats + (lp.list ? 36 : 15); /* chunk counter, zeroed before every launch */
    const long long n_idx = lp.list ? (long long)(u32)uni((int)(u32)stats[35]) : n_chunks;
    /* The queue is one device-scope counter of chunks.  A single address takes
     * on the order of 10^8 atomics per second across the 8 XCDs, which caps
     * scenes of cheap samples (C5: 64-sample chunks at ~85 M/s).  So a wave
     * whose last run of chunks took under PT_GRAB_TICKS (100 MHz ticks) per
     * chunk takes a run of lp.grab chunks per atomic, while more than 8 runs
     * per wave remain; otherwise single chunks.  Built (PT_GRAB_RUNS) and asked
     * for only in lane-walk scenes, whose chunks are uniformly cheap (C5 +53 %); C3's mix
     * of cheap and expensive chunks loses with them (runs of 8 throughout:
     * -6.6 %, adaptive: -0.45 %, profiles/round5/ab_grab_*.txt) and is far from
     * the atomic's rate.  The order of the items changes no result. */
    auto uniform_chunk = [&](long long c) {
        return ((long long)uni((int)(c >> 32)) << 32) | (long long)(u32)uni((int)c);
    };
#if PT_GRAB_RUNS
    const long long nwaves = (long long)gridDim.x * PT_WPW;
    const int GRAB = lp.grab > 1 ? lp.grab : 1;
    int cheap = 0; /* the last run took under PT_GRAB_TICKS per chunk (unknown: single chunks) */
    auto want = [&](long long from) { /* run length of the next request, seen from chunk `from` */
        return (GRAB > 1 && cheap && n_idx - from > 8ll * GRAB * nwaves) ? GRAB : 1;
    };
    auto dequeue = [&](int k) {
        long long c = 0;
        if (lane == 0)
            c = (long long)atomicAdd(work, (u64)k);
        return c;
    };
    int nk = 1, left = 0, cur = 1; /* nk: length of the run `next` starts; left: chunks left in this run */
    long long next = dequeue(nk), run = 0;
    u64 t_run = 0;
#else
    auto dequeue = [&]() {
        long long c = 0;
        if (lane == 0)
            c = (long long)atomicAdd(work, 1ull);
        return c;
    };
    long long next = dequeue();
#endif
#ifdef PT_BAIL_STATS
    pt_bail_flag[blockIdx.x * blockDim.x + threadIdx.x] = 0u;
    u64 bs[6] = {0, 0, 0, 0, 0, 0};
#endif
    for (;;) {
#if PT_GRAB_RUNS
        if (left == 0) {
            run = uniform_chunk(next);
            left = cur = nk;
            t_run = __builtin_amdgcn_s_memrealtime();
#if PT_DEQUEUE_PREFETCH
            /* the next run's dequeue is in flight while this one is traced */
            nk = want(run + left);
            next = dequeue(nk);
#endif
        }
        const long long idx = run++;
        left--;
        if (idx >= n_idx)
            break;
#else
        const long long idx = uniform_chunk(next);
        if (idx >= n_idx)
            break;
#if PT_DEQUEUE_PREFETCH
        /* the next chunk's dequeue is in flight while this one is traced */
        next = dequeue();
#endif
#endif
        const long long chunk = lp.list ? uniform_chunk((long long)lp.list[idx]) : idx;
        const long long item0 = chunk * CH;
        PT_T0(tchunk);
        /* the chunk's camera queries, one per lane */
        CamHit ch = {0, 0.0f, 0u, 0};
        int ldone = 0, lq = 0, lsh = 0;
        int lpix = 0, ls = 0; /* the lane's (pixel, sample), read by the wave loop below */
        V3 lres = mk(0, 0, 0);
        const bool lvalid = lane < CH && item0 + lane < lp.n_items;
        if (lvalid) {
            const long long item = item0 + lane;
            long long slot;
            int s;
            item_slot(lp, item, slot, s);
            const int pix = pixels ? pixels[slot] : (int)slot;
            lpix = pix, ls = s;
            Rng r;
            rng_seed(r, lp.seed, PT_ITEM_KEY(lp, pix), (u64)s);
            typename S::Root::Ctx ctx;
#ifdef PT_RAYS
            /* the caller's ray (pixels == nullptr: pix is the ray's index) */
            const float *rr = lp.rays + 7 * (long long)pix;
            const V3 o = mk(rr[0], rr[1], rr[2]), d = mk(rr[3], rr[4], rr[5]);
            const float str = rr[6];
            S::Root::prep_l(ctx, o, e);
#else
            const V3 o = mk(0, 0, 0), d = camera_dir(lp, pix, r);
            const float str = 1.0f;
            S::Root::prep(ctx, o, e);
#endif
            bool ex = false;
#ifdef PT_LANE_WALK
            if constexpr (LIGHT) {
                bool und;
                ch.hit = lane_first_hit_light<typename S::Root>(ctx, d, e, ch.t, ch.ref, ex, und) ? 1 : 0;
                ch.ex = ex ? 1 : 0;
                ldone = !und && lane_walk<S, true>(e, lp.depth, o, d, str, ch, lres, lq, lsh) ? 1 : 0;
            } else
#endif
            {
            ch.hit = lane_first_hit<typename S::Root>(ctx, d, e, ch.t, ch.ref, ex) ? 1 : 0;
            ch.ex = ex ? 1 : 0;
#if defined(PT_LANE_SCATTER) /* per scene, pt_scene_set_lane_scatter */
            ldone = lane_walk_sc<S, MAXD, STRICT>(e, lp.depth, o, d, str, ch, r, lres, lq, lsh) ? 1 : 0;
#elif defined(PT_LANE_WALK) /* per scene, pt_scene_set_lane_walk */
            ldone = lane_walk<S>(e, lp.depth, o, d, str, ch, lres, lq, lsh) ? 1 : 0;
#else
            ldone = lane_sample<S>(e, lp.depth, o, d, str, ch, lres, lq, lsh) ? 1 : 0;
#endif
            }
        }
        PT_ACC2(cnt, 1, tchunk); /* the lane-parallel front end */
        /* the light kernel leaves a chunk with a lane it could not finish (a
         * query its checks cannot decide, a scatter loop, a deep tree) to the
         * full kernel, whole: a chunk's sums come from one kernel */
        bool bailed = false;
        if constexpr (LIGHT) {
            bailed = __ballot(lvalid && !ldone) != 0ull;
            if (bailed && lane == 0)
                lp.bail[atomicAdd(&stats[35], 1ull)] = (unsigned)chunk;
        }
#ifdef PT_BAIL_STATS
        {
            unsigned &fl = pt_bail_flag[blockIdx.x * blockDim.x + threadIdx.x];
            const u64 BM = __ballot(fl != 0u), BW = __ballot(lvalid && !ldone);
            fl = 0u;
            bs[0]++, bs[1] += BM ? 1 : 0, bs[2] += BW ? 1 : 0, bs[3] += (BM | BW) ? 1 : 0;
            bs[4] += __popcll(BM), bs[5] += __popcll(BW);
        }
#endif
        if (!bailed) {
            /* statistics of the samples finished by their lane */
#if defined(PT_LANE_WALK) || defined(PT_LANE_SCATTER)
            {
                /* per-lane counts: a wave sum of small integers */
                int q = ldone ? lq : 0, h = ldone ? lsh : 0;
#pragma unroll
                for (int w = 32; w >= 1; w >>= 1)
                    q += __shfl_xor(q, w), h += __shfl_xor(h, w);
                cnt.queries += (u64)(u32)uni(q);
                cnt.shaded += (u64)(u32)uni(h);
            }
#else
            const u64 D = __ballot(ldone), Q2 = __ballot(ldone && lq == 2), SH = __ballot(ldone && lsh);
            cnt.queries += (u64)(__popcll(D) + __popcll(Q2));
            cnt.shaded += (u64)__popcll(SH);
#endif
        }
        V3 mine = lres;
        if constexpr (!LIGHT) {
        /* park the lanes' state in LDS for the walks below */
        uint4 *const lb = lbuf[wave];
        const bool lwalk = lvalid && !ldone;
        lb[lane] = lwalk ? make_uint4((u32)lpix, (u32)ls | ((u32)ch.hit << 30) | ((u32)ch.ex << 31),
                                      __float_as_uint(ch.t), ch.ref)
                         : make_uint4(__float_as_uint(lres.x), __float_as_uint(lres.y), __float_as_uint(lres.z), 0u);
        /* the other items, one after another by the whole wave; only this mask
         * stays live across the walks */
        for (u64 todo = __ballot(lwalk); todo; todo &= todo - 1) {
            const int j = uni(__builtin_ctzll(todo));
            PT_T0(tt);
            const uint4 q = lb[j];
            const int qy = uni((int)q.y);
            const CamHit cam = {(qy >> 30) & 1, unif(__uint_as_float(q.z)), (u32)uni((int)q.w), (int)((u32)qy >> 31)};
            V3 c = trace_sample<S, MAXD, STRICT>(e, lp, uni((int)q.x), qy & 0x3FFFFFFF, stk[wave], L, jump, jl, cnt,
                                                 cam);
            PT_ACC(cnt, 6, tt);
            if (lane == j)
                lb[j] = make_uint4(__float_as_uint(c.x), __float_as_uint(c.y), __float_as_uint(c.z), 0u);
        }
        const uint4 mr = lb[lane];
        mine = mk(__uint_as_float(mr.x), __uint_as_float(mr.y), __uint_as_float(mr.z));
        }
        PT_T0(tout);
#if PT_GRAB_RUNS
        if (left == 0) {
            cheap = __builtin_amdgcn_s_memrealtime() - t_run < (u64)PT_GRAB_TICKS * (u64)cur;
#if !PT_DEQUEUE_PREFETCH
            nk = want(run);
            next = dequeue(nk);
#endif
        }
#elif !PT_DEQUEUE_PREFETCH
        next = dequeue();
#endif
        const long long my = item0 + lane;
        if (bailed) {
            /* the full kernel writes this chunk */
        } else if (lp.block_sums) {
            /* the chunk is one 32-sample block of one slot (slot-major, chunk
             * 32, nsamp % 32 == 0): its 32-leaf pairwise tree is the block
             * partial of the fast order's pixel sum.  Level w adds lane
             * k + w into lane k, so lane 0 ends with pt_tree32's association.
             * The three sums are read out of lane 0 here, at full exec, and
             * lanes 0-2 store one channel each: a read of lane 0 inside a
             * lane-conditional branch would let the compiler sink the last
             * level's add into that branch, where lane 0 does not run. */
            V3 b = mine;
#pragma unroll
            for (int w = 1; w < 32; w *= 2) {
                const float ox = __shfl_down(b.x, w), oy = __shfl_down(b.y, w), oz = __shfl_down(b.z, w);
                b = mk(b.x + ox, b.y + oy, b.z + oz);
            }
            /* a 64-item chunk is two blocks: lanes 0-31 and 32-63 (level w <= 16
             * stays inside each half), lane 32 holds the second partial */
            const float bx = rdlane(b.x, 0), by = rdlane(b.y, 0), bz = rdlane(b.z, 0);
            const float cx = rdlane(b.x, 32), cy = rdlane(b.y, 32), cz = rdlane(b.z, 32);
            const float v = lane == 0 ? bx : lane == 1 ? by : lane == 2 ? bz : lane == 3 ? cx : lane == 4 ? cy : cz;
            if (lane < 3 * (CH >> 5))
                out[3 * (item0 >> 5) + lane] = v;
        } else if (lane < CH && my < lp.n_items) {
            long long slot;
            int s;
            item_slot(lp, my, slot, s);
            const long long st = slot * lp.nsamp + (s - lp.s0); /* the stage stays slot-major for pt_reduce */
            out[3 * st + 0] = mine.x;
            out[3 * st + 1] = mine.y;
            out[3 * st + 2] = mine.z;
        }
        PT_ACC2(cnt, 2, tout);
        PT_ACC2(cnt, 0, tchunk);
    }
    if (lane == 0) {
        atomicAdd(&stats[0], cnt.queries);
        atomicAdd(&stats[1], cnt.leaf);
        atomicAdd(&stats[2], cnt.attempts);
        atomicAdd(&stats[3], cnt.rounds);
        atomicAdd(&stats[4], cnt.shaded);
        atomicAdd(&stats[5], cnt.nonleaf);
        atomicAdd(&stats[6], cnt.slow);
        atomicAdd(&stats[7], cnt.dark);
        atomicAdd(&stats[24], cnt.mid);
#ifdef PT_BAIL_STATS /* chunks; with a lane merge; with wave walks; either; lanes merged; lanes walked */
        for (int k = 0; k < 6; k++)
            atomicAdd(&stats[16 + k], bs[k]);
#endif
        const u64 t_end = __builtin_amdgcn_s_memrealtime();
        atomicMax(&stats[26], ~t_start); /* earliest start, complemented */
        atomicMax(&stats[27], t_end);    /* latest end */
        atomicAdd(&stats[28], t_end - t_start);
        atomicAdd(&stats[29], 1ull);
#ifdef PT_PHASE_TIMING
        for (int k = 0; k < 7; k++)
            atomicAdd(&stats[8 + k], cnt.ph[k]);
        for (int k = 0; k < 8; k++)
            atomicAdd(&stats[16 + k], cnt.np[k]);
        atomicAdd(&stats[30], cnt.sp[0]);
        atomicAdd(&stats[25], cnt.ch[0]);
        atomicAdd(&stats[32], cnt.ch[1]);
        atomicAdd(&stats[33], cnt.ch[2]);
        atomicAdd(&stats[31], cnt.sp[1]);
        atomicAdd(&stats[34], cnt.sp[2]);
#endif
    }
}


/* ---- boundary queries (pt_query_spans, pt_tex_eval) -------------------
 * The reference's query virtuals served on the device, one ray / point per
 * lane.  SpanIterator (include/span.h:129-171) of an object: init(ray), then
 * next() until isAtEnd(); every span in the reference's Span form (start,
 * startNormal, startMaterial, end, endNormal, endMaterial; span.h:12-120) --
 * the same lazy merges the render kernel runs, with each normal recomputed
 * from (ray, t, primitive, flip) as the render kernel does for its hit
 * (copyEndFromStart / copyStartFromEnd negate, span.h:100-112).  Ten words per
 * span: t, normal, material (compact index, as int bits) for each end. */
template <class R>
__device__ __forceinline__ void query_spans(const Env &e, const float *__restrict__ rays, long long n, int max_spans,
                                            float *__restrict__ out, int *__restrict__ counts)
{
    const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n)
        return;
    const float *r = rays + 6 * i;
    const V3 o = mk(r[0], r[1], r[2]), d = mk(r[3], r[4], r[5]);
    typename R::Ctx ctx;
    R::prep_l(ctx, o, e);
    typename R::St st;
    R::init(st, ctx, mkray(d), e);
    CS sp;
    int c = 0;
    while (R::pull(st, sp)) {
        if (c < max_spans) {
            V3 n0 = R::normal(ref_prim(sp.r0), sp.t0, o, d, e), n1 = R::normal(ref_prim(sp.r1), sp.t1, o, d, e);
            if (sp.r0 & FLIP)
                n0 = -n0;
            if (sp.r1 & FLIP)
                n1 = -n1;
            float *q = out + ((long long)i * max_spans + c) * 10;
            q[0] = sp.t0, q[1] = n0.x, q[2] = n0.y, q[3] = n0.z, q[4] = __int_as_float(ref_mat(sp.r0));
            q[5] = sp.t1, q[6] = n1.x, q[7] = n1.y, q[8] = n1.z, q[9] = __int_as_float(ref_mat(sp.r1));
        }
        c++;
    }
    counts[i] = c;
}
/* Texture::getColor / getFloat (include/texture.h:13-18) at one point per lane */
template <class T>
__device__ __forceinline__ void tex_eval(const Env &e, const float *__restrict__ pts, long long n,
                                         float *__restrict__ rgb, float *__restrict__ val)
{
    const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n)
        return;
    const V3 p = mk(pts[3 * i], pts[3 * i + 1], pts[3 * i + 2]);
    const V3 c = T::color(p, e);
    rgb[3 * i] = c.x, rgb[3 * i + 1] = c.y, rgb[3 * i + 2] = c.z;
    val[i] = T::value(p, e);
}

} // namespace ptd

#define PT_DEFINE_QUERY(ROOT)                                                                               \
    extern "C" __global__ __launch_bounds__(256) void pt_query_spans(                                      \
        const float *__restrict__ P, const ptd::PtImage *__restrict__ imgs, const float *__restrict__ rays, \
        long long n, int max_spans, float *__restrict__ out, int *__restrict__ counts)                    \
    {                                                                                                       \
        const ptd::Env e = {P, imgs};                                                                       \
        ptd::query_spans<ROOT>(e, rays, n, max_spans, out, counts);                                         \
    }
#define PT_DEFINE_TEXEVAL(TEX)                                                                              \
    extern "C" __global__ __launch_bounds__(256) void pt_tex_eval(                                         \
        const float *__restrict__ P, const ptd::PtImage *__restrict__ imgs, const float *__restrict__ pts,  \
        long long n, float *__restrict__ rgb, float *__restrict__ val)                                     \
    {                                                                                                       \
        const ptd::Env e = {P, imgs};                                                                       \
        ptd::tex_eval<TEX>(e, pts, n, rgb, val);                                                            \
    }

#ifdef PT_MIN_WAVES /* per scene (pt_scene_set_occupancy), never above what LDS admits: a higher
                       cap would only lower the VGPR budget without adding a resident wave */
#define PT_MIN_WG(SCENE, MAXD)                                                                              \
    (PT_MIN_WAVES < ptd::min_workgroups<SCENE, MAXD>() ? PT_MIN_WAVES : ptd::min_workgroups<SCENE, MAXD>())
#else
#define PT_MIN_WG(SCENE, MAXD) (ptd::min_workgroups<SCENE, MAXD>())
#endif

#define PT_RENDER_ARGS                                                                                     \
    const float *__restrict__ P, const ptd::PtImage *__restrict__ imgs, const u64 *__restrict__ jump,      \
        float *__restrict__ out, const int *__restrict__ pixels, u64 *__restrict__ stats, ptd::PtLaunch lp

/* Lane-walk scenes (C5) also get a light kernel for split launches: the
 * chunks whose every lane the lane walk finishes with decided queries (97 % of
 * C5's) at PT_LIGHT_WG workgroups per CU -- no lazy merge, no wave walk, so
 * few registers -- and the rest through the full kernel at its own
 * occupancy.  Same statements on the chunks it finishes: the same bits. */
#ifdef PT_LANE_WALK
#ifndef PT_LIGHT_WG
#define PT_LIGHT_WG 4
#endif
#define PT_DEFINE_LIGHT(SCENE, MAXD)                                                                        \
    extern "C" __global__ __launch_bounds__(64 * PT_WPW, PT_LIGHT_WG) void pt_render_light(PT_RENDER_ARGS)  \
    {                                                                                                       \
        ptd::render_chunk<SCENE, MAXD, false, true>(P, imgs, jump, out, pixels, stats, lp);                \
    }
#else
#define PT_DEFINE_LIGHT(SCENE, MAXD)
#endif

#define PT_DEFINE_KERNELS(SCENE, MAXD)                                                                      \
    PT_DEFINE_LIGHT(SCENE, MAXD)                                                                            \
    extern "C" __global__ __launch_bounds__(64 * PT_WPW, PT_MIN_WG(SCENE, MAXD)) void pt_render_fast(PT_RENDER_ARGS) \
    {                                                                                                       \
        ptd::render_chunk<SCENE, MAXD, false>(P, imgs, jump, out, pixels, stats, lp);                      \
    }                                                                                                       \
    extern "C" __global__ __launch_bounds__(64 * PT_WPW, PT_MIN_WG(SCENE, MAXD)) void pt_render_strict(PT_RENDER_ARGS) \
    {                                                                                                       \
        ptd::render_chunk<SCENE, MAXD, true>(P, imgs, jump, out, pixels, stats, lp);                       \
    }

#endif

#ifndef PT_DEVICE_REDUCE_DEFINED
#define PT_DEVICE_REDUCE_DEFINED
/* Per-pixel sample sums, one thread per pixel slot, carried across passes in
 * accum; on the last pass acc / spp goes to the frame buffer.
 *   mode 0 (reference order): acc = ((acc + x_0) + x_1) + ..., tracePixel's
 *          own accumulation (path-trace.h:192-199), from per-sample values;
 *   mode 1 (fast order, per-sample stage): samples in blocks of 32 from
 *          the call's first sample, each block its 32-leaf pairwise tree
 *          (missing leaves -0.0f), acc = ((acc + B_0) + B_1) + ...;
 *   mode 2 (fast order, block stage): the same with the block partials
 *          already summed by the render kernel (one per 32 samples). */
__device__ __forceinline__ float pt_tree32(const float *v, int n, int stride)
{
    float b[32];
#pragma unroll
    for (int k = 0; k < 32; k++)
        b[k] = k < n ? v[k * stride] : -0.0f;
#pragma unroll
    for (int w = 1; w < 32; w *= 2)
#pragma unroll
        for (int k = 0; k < 32; k += 2 * w)
            b[k] = b[k] + b[k + w];
    return b[0];
}
extern "C" __global__ __launch_bounds__(256) void pt_reduce(const float *__restrict__ in, float *__restrict__ accum,
                                                            float *__restrict__ fb, const int *__restrict__ pixels,
                                                            long long nslots, int nsamp, int first, int last,
                                                            float spp, int mode)
{
    const long long slot = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (slot >= nslots)
        return;
    float ax = 0.0f, ay = 0.0f, az = 0.0f;
    if (!first) {
        ax = accum[3 * slot + 0];
        ay = accum[3 * slot + 1];
        az = accum[3 * slot + 2];
    }
    if (mode == 2) {
        const int nb = nsamp >> 5;
        const float *p = in + 3 * slot * (long long)nb;
        for (int b = 0; b < nb; b++) {
            ax = ax + p[3 * b + 0];
            ay = ay + p[3 * b + 1];
            az = az + p[3 * b + 2];
        }
    } else if (mode == 1) {
        const float *p = in + 3 * slot * (long long)nsamp;
        for (int s = 0; s < nsamp; s += 32) {
            const int n = nsamp - s < 32 ? nsamp - s : 32;
            ax = ax + pt_tree32(p + 3 * s + 0, n, 3);
            ay = ay + pt_tree32(p + 3 * s + 1, n, 3);
            az = az + pt_tree32(p + 3 * s + 2, n, 3);
        }
    } else {
        const float *p = in + 3 * slot * (long long)nsamp;
        for (int s = 0; s < nsamp; s++) {
            ax = ax + p[3 * s + 0];
            ay = ay + p[3 * s + 1];
            az = az + p[3 * s + 2];
        }
    }
    if (last) {
        const long long pix = pixels ? (long long)pixels[slot] : slot;
        fb[3 * pix + 0] = ax / spp;
        fb[3 * pix + 1] = ay / spp;
        fb[3 * pix + 2] = az / spp;
    } else {
        accum[3 * slot + 0] = ax;
        accum[3 * slot + 1] = ay;
        accum[3 * slot + 2] = az;
    }
}
#endif

#ifdef PT_SELFTEST
/* Bitwise check of the exact fast paths (csqrt, cdiv, cnormalize) against the
 * compiler's correctly rounded sqrtf and '/', on n hashed inputs: half drawn
 * from all 2^32 bit patterns, half with exponents around the fast ranges. */
__device__ __forceinline__ float pt_st_float(u64 h, int mode)
{
    u32 b = (u32)h;
    if (mode) {
        u32 e = 40u + (u32)((h >> 32) % 180u); /* biased exponent 40..219 */
        b = (b & 0x807fffffu) | (e << 23);
    }
    return __uint_as_float(b);
}
__device__ __forceinline__ bool pt_st_same(float a, float b)
{
    return __float_as_uint(a) == __float_as_uint(b) || (a != a && b != b);
}
extern "C" __global__ void pt_selftest_math(u64 n, u64 seed, unsigned long long *bad)
{
    unsigned long long bs = 0, bd = 0, bn = 0;
    for (u64 i = (u64)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (u64)gridDim.x * blockDim.x) {
        u64 h1 = ptd::splitmix64(seed ^ (i * 3)), h2 = ptd::splitmix64(seed ^ (i * 3 + 1)),
            h3 = ptd::splitmix64(seed ^ (i * 3 + 2));
        int mode = (int)(i & 1);
        float x = pt_st_float(h1, mode), y = pt_st_float(h2, mode), z = pt_st_float(h3, mode);
        if (!pt_st_same(ptd::csqrt(__builtin_fabsf(x)), __builtin_sqrtf(__builtin_fabsf(x))))
            bs++;
        ptd::Rcp R = ptd::mkrcp(y);
        if (!pt_st_same(ptd::cdiv(x, R, ptd::den_ok(y)), x / y))
            bd++;
        float sc = mode ? 1.0f : 1e-30f;
        ptd::V3 v = ptd::mk(x * sc, y * sc, z * sc);
        ptd::V3 a = ptd::cnormalize(v), b = ptd::normalize(v);
        if (!(pt_st_same(a.x, b.x) && pt_st_same(a.y, b.y) && pt_st_same(a.z, b.z)))
            bn++;
    }
    if (bs)
        atomicAdd(&bad[0], bs);
    if (bd)
        atomicAdd(&bad[1], bd);
    if (bn)
        atomicAdd(&bad[2], bn);
}
/* The restated glibc float libm (libm_atan2f, libm_asinf, libm_logf) on
 * caller operands: out[3i..3i+2] = atan2f(ops[2i], ops[2i+1]),
 * asinf(ops[2i]), logf(ops[2i+1]); the caller compares with its host's glibc
 * (tests/test_libm.py). */
extern "C" __global__ void pt_selftest_libm(const float *ops, u64 n, float *out)
{
    for (u64 i = (u64)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (u64)gridDim.x * blockDim.x) {
        const float y = ops[2 * i], x = ops[2 * i + 1];
        out[3 * i] = ptd::libm_atan2f(y, x);
        out[3 * i + 1] = ptd::libm_asinf(y);
        out[3 * i + 2] = ptd::libm_logf(x);
    }
}
#endif
