/* Exhaustive host check that fma(fma(-q0,180,x),r,q0), q0 = x*r, r = RN(1/180),
 * equals RN(x/180) for every finite float with |x| >= 2^-100 (the trace
 * kernel's div180(); smaller |x| take the IEEE division).  Build:
 *   gcc -O2 -mfma -o /tmp/check_div180 scripts/check_div180.c -lm
 * Result (2026-10-15): tested 3825205248 bad 0. */
#include <math.h>
#include <stdio.h>
#include <stdint.h>
#include <string.h>
int main(void) {
    const float r = 1.0f / 180.0f;
    uint64_t bad = 0, tested = 0;
    for (uint64_t u = 0; u <= 0xFFFFFFFFull; ++u) {
        uint32_t b = (uint32_t)u; float x; memcpy(&x, &b, 4);
        if (!isfinite(x) || fabsf(x) < 0x1p-100f) continue;
        float q = x / 180.0f;
        float q0 = x * r;
        float rem = fmaf(-q0, 180.0f, x);
        float q1 = fmaf(rem, r, q0);
        uint32_t a, c; memcpy(&a, &q, 4); memcpy(&c, &q1, 4);
        ++tested;
        if (a != c) { if (bad < 5) printf("bad x=%a q=%a q1=%a\n", x, q, q1); ++bad; }
    }
    printf("tested %llu bad %llu\n", (unsigned long long)tested, (unsigned long long)bad);
    return 0;
}
