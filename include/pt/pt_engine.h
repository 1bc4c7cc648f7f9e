/*
 * pt_engine.h -- the per-(pixel, sample) random engine of the MI355X renderer.
 *
 * The reference threads a caller-supplied engine type `T` through
 * tracePixel<T>/traceRay<T> (reference include/path-trace.h:58-59, :187-188)
 * and only requires `unsigned operator()()`, `static min()`, `static max()`
 * (consumed by uniform_real_distribution, include/vector3d.h:14-34).  Its own
 * DefaultRandomEngine (include/path-trace.h:21-54) is one global, racy LCG
 * whose 32-bit seed() gives adjacent seeds nearly identical streams, so it
 * cannot give per-sample reproducibility.  This header keeps the reference
 * engine's RECURRENCE and output exactly and only replaces its seeding:
 *
 *   v' = 214013 * v + 2531011  (mod 2^64),  output = (unsigned)(v' >> 32)
 *     (DefaultRandomEngine::operator(), include/path-trace.h:45-49)
 *
 * with a private starting state per (pixel, sample):
 *   key = splitmix64(run_seed) ^ (pixel_index << 20) ^ sample_index
 *   v   = splitmix64(key)
 * pixel_index = y * width + x over the WHOLE frame, so a pixel's samples are
 * identical no matter which GPU / tile / pass renders them.  Every stream is
 * a window of the reference's one sequence, at a hashed 64-bit offset.
 *
 * The GPU evaluates a scatter loop's rejection attempts 64 at a time (one
 * attempt per lane) and must know the state 3*l draws ahead for lane l; an LCG
 * jumps k steps in O(1):
 *   v_{n+k} = A_k * v_n + G_k * c,  A_k = M^k,  G_k = sum_{j<k} M^j.
 * `inc` (= c) is kept in the engine state so the jump formula is explicit.
 */
#ifndef PT_ENGINE_H
#define PT_ENGINE_H

#include <stdint.h>

#if defined(__HIPCC__) || defined(__HIPCC_RTC__)
#define PT_HD __host__ __device__ inline
#else
#define PT_HD static inline
#endif

#define PT_LCG_MULT 214013ULL  /* include/path-trace.h:47 */
#define PT_LCG_INC 2531011ULL  /* include/path-trace.h:47 */
#define PT_SPLITMIX_GAMMA 0x9E3779B97F4A7C15ULL

PT_HD uint64_t pt_splitmix64(uint64_t x)
{
    uint64_t z = x + PT_SPLITMIX_GAMMA;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    return z ^ (z >> 31);
}

/* DefaultRandomEngine::operator()'s output of the UPDATED state */
PT_HD uint32_t pt_lcg_output(uint64_t updated) { return (uint32_t)(updated >> 32); }

PT_HD uint64_t pt_sample_key(uint64_t run_seed, uint64_t pixel_index, uint64_t sample_index)
{
    return pt_splitmix64(run_seed) ^ (pixel_index << 20) ^ sample_index;
}

PT_HD void pt_engine_seed(uint64_t key, uint64_t *state, uint64_t *inc)
{
    *state = pt_splitmix64(key);
    *inc = PT_LCG_INC;
}

/* (A_k, G_k) of the jump state_{n+k} = A_k*state_n + G_k*inc. */
PT_HD void pt_lcg_jump_coeffs(uint32_t k, uint64_t *a_out, uint64_t *g_out)
{
    uint64_t a = 1, g = 0, m = PT_LCG_MULT, h = 1; /* h = sum_{j<2^i} M^j for current power m = M^(2^i) */
    while (k) {
        if (k & 1u) {
            /* apply block of size 2^i: (a, g) <- (m*a, m*g + h) */
            g = g * m + h;
            a = a * m;
        }
        h = h * (m + 1);
        m = m * m;
        k >>= 1;
    }
    *a_out = a;
    *g_out = g;
}

#ifdef __cplusplus
#if defined(__HIPCC__) || defined(__HIPCC_RTC__)
#define PT_HDM __host__ __device__
#else
#define PT_HDM
#endif
/* The engine type plugged into the reference's `T` slot
 * (unsigned operator()(), static min(), static max()). */
struct PtSampleEngine
{
    uint64_t state, inc;
    PT_HDM PtSampleEngine() : state(0), inc(1) {}
    PT_HDM PtSampleEngine(uint64_t run_seed, uint64_t pixel_index, uint64_t sample_index)
    {
        pt_engine_seed(pt_sample_key(run_seed, pixel_index, sample_index), &state, &inc);
    }
    PT_HDM static unsigned min() { return 0; }
    PT_HDM static unsigned max() { return 0xFFFFFFFFu; }
    PT_HDM unsigned operator()()
    {
        state = state * PT_LCG_MULT + inc;
        return pt_lcg_output(state);
    }
    PT_HDM void discard(uint64_t k)
    {
        while (k) {
            uint32_t step = k > 0xFFFFFFFFull ? 0xFFFFFFFFu : (uint32_t)k;
            uint64_t a, g;
            pt_lcg_jump_coeffs(step, &a, &g);
            state = a * state + g * inc;
            k -= step;
        }
    }
};
#endif

#endif
