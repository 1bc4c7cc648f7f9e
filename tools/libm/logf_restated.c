/* glibc 2.35 logf restated (the device's libm_logf, pt_device.h) and checked
 * against this host's glibc logf on every non-negative float.
 *
 * Algorithm and constants: glibc sysdeps/ieee754/flt-32/e_logf.c and
 * e_logf_data.c, contributed by Szabolcs Nagy from ARM's optimized-routines
 * (Copyright (c) 2017-2018 Arm Ltd., SPDX-License-Identifier: MIT; in glibc
 * under LGPL-2.1-or-later).  Restated for bit parity with the reference's
 * LogTexture (include/filter_texture.h:62-67: std::log on a float = logf).
 *
 * glibc selects FMA-compiled variants of logf at run time on FMA hosts, so
 * the check runs the double arithmetic both ways (mode 0: separate multiply
 * and add, as the device compiles it with -ffp-contract=off; mode 15: every
 * multiply-add fused) and both must agree with glibc.
 *   gcc -O2 -ffp-contract=off tools/libm/logf_restated.c -lm && ./a.out
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <stdio.h>
#include <string.h>

static inline uint32_t asu(float f) { uint32_t i; memcpy(&i, &f, 4); return i; }
static inline float asf(uint32_t i) { float f; memcpy(&f, &i, 4); return f; }
static const double T[16][2] = {
    {0x1.661ec79f8f3bep+0, -0x1.57bf7808caadep-2}, {0x1.571ed4aaf883dp+0, -0x1.2bef0a7c06ddbp-2},
    {0x1.49539f0f010bp+0, -0x1.01eae7f513a67p-2},  {0x1.3c995b0b80385p+0, -0x1.b31d8a68224e9p-3},
    {0x1.30d190c8864a5p+0, -0x1.6574f0ac07758p-3}, {0x1.25e227b0b8eap+0, -0x1.1aa2bc79c81p-3},
    {0x1.1bb4a4a1a343fp+0, -0x1.a4e76ce8c0e5ep-4}, {0x1.12358f08ae5bap+0, -0x1.1973c5a611cccp-4},
    {0x1.0953f419900a7p+0, -0x1.252f438e10c1ep-5}, {0x1p+0, 0x0p+0},
    {0x1.e608cfd9a47acp-1, 0x1.aa5aa5df25984p-5},  {0x1.ca4b31f026aap-1, 0x1.c5e53aa362eb4p-4},
    {0x1.b2036576afce6p-1, 0x1.526e57720db08p-3},  {0x1.9c2d163a1aa2dp-1, 0x1.bc2860d22477p-3},
    {0x1.886e6037841edp-1, 0x1.1058bc8a07ee1p-2},  {0x1.767dcf5534862p-1, 0x1.4043057b6ee09p-2},
};
static const double Ln2 = 0x1.62e42fefa39efp-1;
static const double A[3] = {-0x1.00ea348b88334p-2, 0x1.5575b0be00b6ap-2, -0x1.ffffef20a4123p-2};

static float my_logf(float x, int fused)
{
    uint32_t ix = asu(x), iz, tmp;
    int k, i;
    double z, r, r2, y, y0, invc, logc;
    if (ix == 0x3f800000)
        return 0;
    if (ix - 0x00800000 >= 0x7f800000 - 0x00800000) {
        if (ix * 2 == 0)
            return -INFINITY;
        if (ix == 0x7f800000)
            return x;
        if ((ix & 0x80000000) || ix * 2 >= 0xff000000)
            return NAN;
        ix = asu(x * 0x1p23f);
        ix -= 23 << 23;
    }
    tmp = ix - 0x3f330000;
    i = (tmp >> (23 - 4)) % 16;
    k = (int32_t)tmp >> 23;
    iz = ix - (tmp & 0x1ffu << 23);
    invc = T[i][0];
    logc = T[i][1];
    z = (double)asf(iz);
    r = fused ? fma(z, invc, -1.0) : z * invc - 1;
    y0 = fused ? fma((double)k, Ln2, logc) : logc + (double)k * Ln2;
    r2 = r * r;
    y = fused ? fma(A[1], r, A[2]) : A[1] * r + A[2];
    y = fused ? fma(A[0], r2, y) : A[0] * r2 + y;
    y = fused ? fma(y, r2, y0 + r) : y * r2 + (y0 + r);
    return (float)y;
}

int main(int argc, char **argv)
{
    /* optional stride: every k-th non-negative float (the test suite's quick form) */
    const uint64_t step = argc > 1 ? strtoull(argv[1], NULL, 10) : 1;
    long bad[2] = {0, 0};
    for (uint64_t u = 0; u < 0x80000000ull; u += step ? step : 1) {
        const float x = asf((uint32_t)u), g = logf(x);
        for (int f = 0; f < 2; f++) {
            const float m = my_logf(x, f);
            if (asu(m) != asu(g) && !(m != m && g != g)) {
                if (bad[f] < 5)
                    printf("mismatch (fused %d) x=%a mine=%a glibc=%a\n", f, x, m, g);
                bad[f]++;
            }
        }
    }
    printf("logf restated vs glibc on every %llu-th of the 2^31 non-negative floats: %ld mismatches (separate), "
           "%ld (fused)\n", (unsigned long long)(step ? step : 1), bad[0], bad[1]);
    return bad[0] || bad[1];
}
