/* fdlibm float atan / atan2 restated (the device's libm_atanf / libm_atan2f,
 * pt_device.h) and checked against this host's glibc 2.35 atanf / atan2f.
 *
 * Algorithm and constants: Sun fdlibm s_atan.c / e_atan2.c as converted to
 * float (e_atan2f.c, s_atanf.c) and shipped in glibc sysdeps/ieee754/flt-32:
 *   Copyright (C) 1993 by Sun Microsystems, Inc. All rights reserved.
 *   Developed at SunPro, a Sun Microsystems, Inc. business.
 *   Permission to use, copy, modify, and distribute this software is freely
 *   granted, provided that this notice is preserved.
 *   (Conversion to float by Ian Lance Taylor, Cygnus Support.)
 *   gcc -O2 -ffp-contract=off tools/libm/atan2f_restated.c -lm && ./a.out */
#include <math.h>
#include <stdio.h>
#include <stdint.h>
#include <string.h>
static inline int32_t bits(float f) { int32_t i; memcpy(&i, &f, 4); return i; }
static const float atanhi[] = {4.6364760399e-01f, 7.8539812565e-01f, 9.8279368877e-01f, 1.5707962513e+00f};
static const float atanlo[] = {5.0121582440e-09f, 3.7748947079e-08f, 3.4473217170e-08f, 7.5497894159e-08f};
static const float aT[] = {3.3333334327e-01f, -2.0000000298e-01f, 1.4285714924e-01f, -1.1111110449e-01f,
                           9.0908870101e-02f, -7.6918758452e-02f, 6.6610731184e-02f, -5.8335702866e-02f,
                           4.9768779427e-02f, -3.6531571299e-02f, 1.6285819933e-02f};
static float my_atanf(float x) {
    int32_t hx = bits(x), ix = hx & 0x7fffffff; int id;
    if (ix >= 0x4c000000) { if (ix > 0x7f800000) return x + x; return hx > 0 ? atanhi[3] + atanlo[3] : -atanhi[3] - atanlo[3]; }
    if (ix < 0x3ee00000) { if (ix < 0x31000000) return x; id = -1; }
    else {
        x = fabsf(x);
        if (ix < 0x3f980000) {
            if (ix < 0x3f300000) { id = 0; x = (2.0f * x - 1.0f) / (2.0f + x); }
            else { id = 1; x = (x - 1.0f) / (x + 1.0f); }
        } else {
            if (ix < 0x401c0000) { id = 2; x = (x - 1.5f) / (1.0f + 1.5f * x); }
            else { id = 3; x = -1.0f / x; }
        }
    }
    float z = x * x, w = z * z;
    float s1 = z * (aT[0] + w * (aT[2] + w * (aT[4] + w * (aT[6] + w * (aT[8] + w * aT[10])))));
    float s2 = w * (aT[1] + w * (aT[3] + w * (aT[5] + w * (aT[7] + w * aT[9]))));
    if (id < 0) return x - x * (s1 + s2);
    z = atanhi[id] - ((x * (s1 + s2) - atanlo[id]) - x);
    return hx < 0 ? -z : z;
}
static const float pi_o_4 = 7.8539818525e-01f, pi_o_2 = 1.5707963705e+00f, pi = 3.1415927410e+00f, pi_lo = -8.7422776573e-08f;
static float my_atan2f(float y, float x) {
    int32_t hx = bits(x), ix = hx & 0x7fffffff, hy = bits(y), iy = hy & 0x7fffffff;
    if (ix > 0x7f800000 || iy > 0x7f800000) return x + y;
    if (hx == 0x3f800000) return my_atanf(y);
    int m = ((hy >> 31) & 1) | ((hx >> 30) & 2);
    if (iy == 0) { switch (m) { case 0: case 1: return y; case 2: return pi; default: return -pi; } }
    if (ix == 0) return hy < 0 ? -pi_o_2 : pi_o_2;
    if (ix == 0x7f800000) {
        if (iy == 0x7f800000) { switch (m) { case 0: return pi_o_4; case 1: return -pi_o_4; case 2: return 3.0f * pi_o_4; default: return -3.0f * pi_o_4; } }
        switch (m) { case 0: return 0.0f; case 1: return -0.0f; case 2: return pi; default: return -pi; }
    }
    if (iy == 0x7f800000) return hy < 0 ? -pi_o_2 : pi_o_2;
    int k = (iy - ix) >> 23; float z;
    if (k > 60) z = pi_o_2 + 0.5f * pi_lo;      /* glibc flt-32: 60, and no m &= 1 (FreeBSD: 26, m &= 1) */
    else if (k < -60 && hx < 0) z = 0.0f;
    else z = my_atanf(fabsf(y / x));
    switch (m) { case 0: return z; case 1: return -z; case 2: return pi - (z - pi_lo); default: return (z - pi_lo) - pi; }
}
static uint64_t s = 0x9E3779B97F4A7C15ull;
static double u(void) { s ^= s << 13; s ^= s >> 7; s ^= s << 17; return (s >> 11) * 0x1p-53; }
int main(void) {
    long n = 20000000, ba = 0, bt = 0;
    for (long i = 0; i < n; i++) {
        float x = (float)(2 * u() - 1), y = (float)(2 * u() - 1);
        if (my_atan2f(y, x) != atan2f(y, x)) { if (ba < 5) printf("atan2f mismatch y=%a x=%a mine=%a glibc=%a\n", y, x, my_atan2f(y, x), atan2f(y, x)); ba++; }
        float t = (float)(8 * u() - 4);
        if (my_atanf(t) != atanf(t)) bt++;
    }
    printf("atan2f mismatches %ld of %ld, atanf %ld\n", ba, n, bt);
    /* the branches uniform operands in [-1, 1] miss: large exponent gaps both
     * ways (k > 26, k < -26 with x < 0), signed zeros, infinities, NaN */
    long be = 0, ne = 0;
    const float mant[] = {1.0f, 1.5f, 1.25f, 1.9999999f, 1.3333334f};
    for (int ey = -140; ey <= 127; ey++)
        for (int ex = -140; ex <= 127; ex += 3)
            for (int a = 0; a < 5; a++)
                for (int b = 0; b < 5; b++)
                    for (int sg = 0; sg < 4; sg++) {
                        float y = ldexpf(mant[a], ey), x = ldexpf(mant[b], ex);
                        if (sg & 1) y = -y;
                        if (sg & 2) x = -x;
                        float m = my_atan2f(y, x), g = atan2f(y, x);
                        ne++;
                        if (bits(m) != bits(g)) { if (be < 5) printf("edge mismatch y=%a x=%a mine=%a glibc=%a\n", y, x, m, g); be++; }
                    }
    const float sp[] = {0.0f, -0.0f, 1.0f, -1.0f, 0x1p-30f, -0x1p-30f, 0x1p-149f, -0x1p-149f, INFINITY, -INFINITY, NAN};
    for (int i = 0; i < 11; i++)
        for (int j = 0; j < 11; j++) {
            float m = my_atan2f(sp[i], sp[j]), g = atan2f(sp[i], sp[j]);
            ne++;
            if (bits(m) != bits(g) && !(m != m && g != g)) { if (be < 10) printf("special mismatch y=%a x=%a mine=%a glibc=%a\n", sp[i], sp[j], m, g); be++; }
        }
    printf("atan2f edge operands: %ld mismatches of %ld\n", be, ne);
    return (ba || bt || be) ? 1 : 0;
}
