#include <math.h>
#include <stdio.h>
#include <stdint.h>
static uint64_t s = 0x9E3779B97F4A7C15ull;
static double u(void) { s ^= s << 13; s ^= s >> 7; s ^= s << 17; return (s >> 11) * 0x1p-53; }
int main(void) {
    long n = 20000000, ba = 0, bs = 0;
    for (long i = 0; i < n; i++) {
        float x = (float)(2 * u() - 1), y = (float)(2 * u() - 1), z = (float)(2 * u() - 1);
        float a = atan2f(y, x), ad = (float)atan2((double)y, (double)x);
        float b = asinf(z), bd = (float)asin((double)z);
        ba += a != ad; bs += b != bd;
    }
    printf("atan2f != (float)atan2: %ld of %ld (%.2e); asinf != (float)asin: %ld (%.2e)\n", ba, n, (double)ba / n, bs, (double)bs / n);
}
