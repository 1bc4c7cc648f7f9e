/* fdlibm float asin restated (the device's libm_asinf, pt_device.h) and
 * checked against this host's glibc 2.35 asinf on every float in [-1, 1].
 * Algorithm and constants: Sun fdlibm e_asin.c as converted to float and
 * shipped in glibc sysdeps/ieee754/flt-32/e_asinf.c:
 *   Copyright (C) 1993 by Sun Microsystems, Inc. All rights reserved.
 *   Developed at SunPro, a Sun Microsystems, Inc. business.
 *   Permission to use, copy, modify, and distribute this software is freely
 *   granted, provided that this notice is preserved.
 *   (Conversion to float by Ian Lance Taylor, Cygnus Support.)
 *   gcc -O2 -ffp-contract=off tools/libm/asinf_restated.c -lm && ./a.out */
#include <math.h>
#include <stdio.h>
#include <stdint.h>
#include <string.h>
static inline int32_t bits(float f) { int32_t i; memcpy(&i, &f, 4); return i; }
static inline float fromb(int32_t i) { float f; memcpy(&f, &i, 4); return f; }
static const float pio2_hi = 1.57079637050628662109375f, pio2_lo = -4.37113900018624283e-8f,
                   pio4_hi = 0.785398185253143310546875f, p0 = 1.666675248e-1f, p1 = 7.495297643e-2f,
                   p2 = 4.547037598e-2f, p3 = 2.417951451e-2f, p4 = 4.216630880e-2f;
static float my_asinf(float x) {
    int32_t hx = bits(x), ix = hx & 0x7fffffff; float t, w, p, q, c, r, s;
    if (ix == 0x3f800000) return x * pio2_hi + x * pio2_lo;
    if (ix > 0x3f800000) return (x - x) / (x - x);
    if (ix < 0x3f000000) {
        if (ix < 0x32000000) return x;
        t = x * x; w = t * (p0 + t * (p1 + t * (p2 + t * (p3 + t * p4)))); return x + x * w;
    }
    w = 1.0f - fabsf(x); t = w * 0.5f;
    p = t * (p0 + t * (p1 + t * (p2 + t * (p3 + t * p4))));
    s = sqrtf(t);
    if (ix >= 0x3F79999A) t = pio2_hi - (2.0f * (s + s * p) - pio2_lo);
    else {
        w = fromb(bits(s) & 0xfffff000);
        c = (t - w * w) / (s + w); r = p;
        p = 2.0f * s * r - (pio2_lo - 2.0f * c); q = pio4_hi - 2.0f * w; t = pio4_hi - (p - q);
    }
    return hx > 0 ? t : -t;
}
static uint64_t s = 0x9E3779B97F4A7C15ull;
static double u(void) { s ^= s << 13; s ^= s >> 7; s ^= s << 17; return (s >> 11) * 0x1p-53; }
int main(void) {
    long n = 20000000, b = 0;
    for (long i = 0; i < n; i++) {
        float z = (float)(2 * u() - 1);
        if (i & 1) z = fromb((bits(z) & 0x807fffff) | 0x3f000000); /* |z| in [0.5, 1) */
        if (my_asinf(z) != asinf(z)) { if (b < 5) printf("mismatch z=%a mine=%a glibc=%a\n", z, my_asinf(z), asinf(z)); b++; }
    }
    /* every float in [-1, 1] */
    long e = 0, tot = 0;
    for (uint32_t i = 0; i <= 0x3f800000u; i++) { float z = fromb((int32_t)i); tot += 2; e += my_asinf(z) != asinf(z); e += my_asinf(-z) != asinf(-z); }
    printf("asinf mismatches %ld of %ld random, %ld of %ld exhaustive\n", b, n, e, tot);
    return (b || e) ? 1 : 0;
}
