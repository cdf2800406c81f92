/* The device restatement of glibc 2.35 sinf / cosf (glibc_sinf / glibc_cosf
 * in opencl-ray-tracer_amd/csrc/rt_scene_device.hip, host-compiled behind
 * rt_debug_glibc_sincosf) against this host's libm on EVERY float: finite
 * values must match bit for bit, inf / NaN inputs must give NaN on both.
 * Needs an FMA-capable x86-64 CPU (glibc then runs __sinf_fma / __cosf_fma,
 * the variant the restatement follows; the non-FMA build differs on 12 sinf
 * and 22 cosf inputs below 120 in magnitude).
 *   gcc -O2 -fopenmp -I include -o /tmp/check_glibc_sincosf scripts/check_glibc_sincosf.c \
 *       -L opencl-ray-tracer_amd -lrt_hip -Wl,-rpath,$PWD/opencl-ray-tracer_amd -lm
 * Result on the build container (2026-10, glibc 2.35): 4278190080 finite
 * floats, 0 sinf and 0 cosf differences; 16777216 inf/NaN inputs all NaN. */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "rt_hip_debug.h"

int main(void) {
    const int64_t kChunk = 1 << 20;
    unsigned long long n_fin = 0, n_nan = 0, bad_s = 0, bad_c = 0, bad_nan = 0;
#pragma omp parallel for reduction(+ : n_fin, n_nan, bad_s, bad_c, bad_nan) schedule(dynamic, 1)
    for (int64_t blk = 0; blk < ((int64_t)1 << 32) / kChunk; ++blk) {
        float* x = malloc(sizeof(float) * kChunk * 3);
        float *s = x + kChunk, *c = s + kChunk;
        for (int64_t i = 0; i < kChunk; ++i) {
            const uint32_t u = (uint32_t)(blk * kChunk + i);
            memcpy(&x[i], &u, 4);
        }
        rt_debug_glibc_sincosf(x, kChunk, s, c);
        for (int64_t i = 0; i < kChunk; ++i) {
            const float rs = sinf(x[i]), rc = cosf(x[i]);
            if (isfinite(x[i])) {
                ++n_fin;
                bad_s += memcmp(&rs, &s[i], 4) != 0;
                bad_c += memcmp(&rc, &c[i], 4) != 0;
            } else {
                ++n_nan;
                bad_nan += !(isnan(s[i]) && isnan(c[i]) && isnan(rs) && isnan(rc));
            }
        }
        free(x);
    }
    printf("finite floats %llu: sinf differences %llu, cosf differences %llu; "
           "inf/NaN inputs %llu, not NaN on both %llu\n", n_fin, bad_s, bad_c, n_nan, bad_nan);
    return (bad_s || bad_c || bad_nan) ? 1 : 0;
}
