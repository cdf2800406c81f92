/* Why the device scene build restates glibc instead
 * of using a device libm: Cube::rotate (Cube.cpp:53-64) takes glm::rotate's
 * cos/sin of float angles, i.e. glibc cosf/sinf, and those are not
 * correctly rounded.  This counts the floats in [-8, 8] where they differ
 * from the correctly rounded (float)sin((double)x), which is all a correctly
 * rounded device libm could give.  The restatement that does match is
 * checked by scripts/check_glibc_sincosf.c.
 *   gcc -O2 -ffp-contract=off -o check_glibc_sincos check_glibc_sincos.c -lm */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>

int main(void) {
    uint64_t n = 0, bad_sin = 0, bad_cos = 0;
    for (int sign = 0; sign < 2; ++sign) {
        for (uint32_t b = 0; b < 0x7f800000u; ++b) {
            const uint32_t u = b | (sign ? 0x80000000u : 0u);
            float x;
            memcpy(&x, &u, 4);
            if (fabsf(x) > 8.0f) break;
            const float s = sinf(x), c = cosf(x);
            const float s2 = (float)sin((double)x), c2 = (float)cos((double)x);
            bad_sin += memcmp(&s, &s2, 4) != 0;
            bad_cos += memcmp(&c, &c2, 4) != 0;
            ++n;
        }
    }
    printf("floats in [-8, 8]: %llu; sinf != RN(sin): %llu; cosf != RN(cos): %llu\n",
           (unsigned long long)n, (unsigned long long)bad_sin, (unsigned long long)bad_cos);
    return 0;
}
