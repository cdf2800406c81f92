// Exhaustive check over every non-negative float x (bit patterns
// 0x00000000 .. 0x7f800000): is (float)v_sqrt_f64((double)x) equal to the
// correctly rounded sqrtf(x)?  (And, for reference, the raw v_sqrt_f32.)
// Build: hipcc --offload-arch=gfx950 -O3 -fhip-fp32-correctly-rounded-divide-sqrt
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ void check(unsigned long long* bad64, unsigned long long* bad32, unsigned* first64) {
    const unsigned n = 0x7f800001u;
    for (unsigned i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
        const float x = __builtin_bit_cast(float, i);
        const float ref = sqrtf(x);  // correctly rounded (build flag)
        const float c64 = (float)__builtin_amdgcn_sqrt((double)x);
        const float c32 = __builtin_amdgcn_sqrtf(x);
        if (__builtin_bit_cast(unsigned, c64) != __builtin_bit_cast(unsigned, ref)) {
            atomicAdd(bad64, 1ull);
            atomicMin(first64, i);
        }
        if (__builtin_bit_cast(unsigned, c32) != __builtin_bit_cast(unsigned, ref))
            atomicAdd(bad32, 1ull);
    }
}

int main() {
    unsigned long long* d;
    unsigned* f;
    hipMalloc(&d, 16);
    hipMalloc(&f, 4);
    hipMemset(d, 0, 16);
    hipMemset(f, 0xff, 4);
    check<<<4096, 256>>>(d, d + 1, f);
    unsigned long long h[2];
    unsigned hf;
    hipMemcpy(h, d, 16, hipMemcpyDeviceToHost);
    hipMemcpy(&hf, f, 4, hipMemcpyDeviceToHost);
    printf("inputs %u  f64-route mismatches %llu (first 0x%08x)  raw f32 mismatches %llu\n",
           0x7f800001u, h[0], hf, h[1]);
    return h[0] == 0 ? 0 : 1;
}
