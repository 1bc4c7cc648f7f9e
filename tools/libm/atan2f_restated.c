/* fdlibm-style float atan / atan2 restated (feasibility check against glibc 2.35) */
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
    if (ix == 0x7f800000) { /* not needed for unit vectors */ return atan2f(y, x); }
    if (iy == 0x7f800000) return hy < 0 ? -pi_o_2 : pi_o_2;
    int k = (iy - ix) >> 23; float z;
    if (k > 26) { z = pi_o_2 + 0.5f * pi_lo; m &= 1; }
    else if (k < -26 && hx < 0) z = 0.0f;
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
}
