/*
 * pt_engine.h -- the per-(pixel, sample) random engine of the MI355X renderer.
 *
 * The reference threads a caller-supplied engine type `T` through
 * tracePixel<T>/traceRay<T> (reference include/path-trace.h:58-59, :187-188)
 * and only requires `unsigned operator()()`, `static min()`, `static max()`
 * (consumed by uniform_real_distribution, include/vector3d.h:14-34).  Its own
 * DefaultRandomEngine (include/path-trace.h:21-54) is one global, racy LCG
 * whose streams for adjacent seeds are nearly identical, so it cannot give
 * per-sample reproducibility.  This header defines the engine that the GPU
 * megakernel, the CPU oracle and the golden generator all plug into `T`:
 *
 *   PCG32 (XSH-RR 64/32).  state' = state * PT_PCG_MULT + inc (mod 2^64);
 *   output = rotr32(((old ^ (old >> 18)) >> 27), old >> 59).
 *
 * Each (pixel, sample) owns a private stream:
 *   key   = splitmix64(run_seed) ^ (pixel_index << 20) ^ sample_index
 *   state = splitmix64(key)
 *   inc   = (splitmix64(key ^ PT_STREAM_SALT) << 1) | 1
 * pixel_index = y * width + x over the WHOLE frame, so a pixel's samples are
 * identical no matter which GPU / tile / pass renders them.
 *
 * Why PCG and not xoroshiro: the GPU evaluates a scatter loop's rejection
 * attempts 64 at a time (one attempt per lane) and must know the engine state
 * 3*l draws ahead for lane l.  An LCG core jumps k steps in O(1):
 *   state_{n+k} = A_k * state_n + G_k * inc,  A_k = M^k,  G_k = sum_{j<k} M^j,
 * while xoroshiro needs a 128x128 GF(2) matrix-vector product per jump.
 * Per-sample increments make every stream a distinct sequence (no overlap).
 */
#ifndef PT_ENGINE_H
#define PT_ENGINE_H

#include <stdint.h>

#if defined(__HIPCC__) || defined(__HIPCC_RTC__)
#define PT_HD __host__ __device__ inline
#else
#define PT_HD static inline
#endif

#define PT_PCG_MULT 6364136223846793005ULL
#define PT_STREAM_SALT 0xD1B54A32D192ED03ULL
#define PT_SPLITMIX_GAMMA 0x9E3779B97F4A7C15ULL

PT_HD uint64_t pt_splitmix64(uint64_t x)
{
    uint64_t z = x + PT_SPLITMIX_GAMMA;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    return z ^ (z >> 31);
}

PT_HD uint32_t pt_pcg_output(uint64_t old)
{
    uint32_t xs = (uint32_t)(((old >> 18) ^ old) >> 27);
    uint32_t rot = (uint32_t)(old >> 59);
    return (xs >> rot) | (xs << ((32u - rot) & 31u));
}

PT_HD uint64_t pt_sample_key(uint64_t run_seed, uint64_t pixel_index, uint64_t sample_index)
{
    return pt_splitmix64(run_seed) ^ (pixel_index << 20) ^ sample_index;
}

PT_HD void pt_engine_seed(uint64_t key, uint64_t *state, uint64_t *inc)
{
    *state = pt_splitmix64(key);
    *inc = (pt_splitmix64(key ^ PT_STREAM_SALT) << 1) | 1ULL;
}

/* (A_k, G_k) of the jump state_{n+k} = A_k*state_n + G_k*inc. */
PT_HD void pt_pcg_jump_coeffs(uint32_t k, uint64_t *a_out, uint64_t *g_out)
{
    uint64_t a = 1, g = 0, m = PT_PCG_MULT, h = 1; /* h = sum_{j<2^i} M^j for current power m = M^(2^i) */
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
        uint64_t old = state;
        state = old * PT_PCG_MULT + inc;
        return pt_pcg_output(old);
    }
    PT_HDM void discard(uint64_t k)
    {
        while (k) {
            uint32_t step = k > 0xFFFFFFFFull ? 0xFFFFFFFFu : (uint32_t)k;
            uint64_t a, g;
            pt_pcg_jump_coeffs(step, &a, &g);
            state = a * state + g * inc;
            k -= step;
        }
    }
};
#endif

#endif
