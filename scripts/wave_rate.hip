// Wave launch rate: 65536 one-wave workgroups (the trace grid at config 3),
// each spinning for a fixed time on s_memrealtime (10 ns ticks) and writing
// one dword; total time vs spin length.  Also 32768 two-wave workgroups.
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ void __launch_bounds__(64) spin1(int* out, unsigned ticks) {
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    while (__builtin_amdgcn_s_memrealtime() - t0 < ticks) __builtin_amdgcn_s_sleep(1);
    if (threadIdx.x == 0) out[blockIdx.x] = 1;
}
__global__ void __launch_bounds__(128) spin2(int* out, unsigned ticks) {
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    while (__builtin_amdgcn_s_memrealtime() - t0 < ticks) __builtin_amdgcn_s_sleep(1);
    if ((threadIdx.x & 63) == 0) out[blockIdx.x * 2 + (threadIdx.x >> 6)] = 1;
}

int main() {
    int* out;
    hipMalloc(&out, 65536 * sizeof(int));
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    for (int round = 0; round < 2; ++round)
        for (unsigned ticks : {0u, 50u, 100u, 200u, 300u, 400u, 600u}) {
            for (int kind = 0; kind < 2; ++kind) {
                auto go = [&] {
                    if (kind == 0) spin1<<<65536, 64>>>(out, ticks);
                    else spin2<<<32768, 128>>>(out, ticks);
                };
                for (int w = 0; w < 3; ++w) go();
                hipDeviceSynchronize();
                hipEventRecord(a);
                const int reps = 20;
                for (int r = 0; r < reps; ++r) go();
                hipEventRecord(b);
                hipEventSynchronize(b);
                float ms;
                hipEventElapsedTime(&ms, a, b);
                const double us = ms * 1e3 / reps;
                std::printf("%s spin %4.1f us: %7.2f us per grid, %.2f waves/ns\n",
                            kind == 0 ? "1-wave WGs" : "2-wave WGs", ticks / 100.0, us,
                            65536.0 / (us * 1e3));
            }
        }
    return 0;
}
