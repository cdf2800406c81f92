// Cost of dependent kernel boundaries on one stream: a 268 MB streaming
// store kernel (the frame write) alone, and preceded by one or two small
// dependent kernels (empty, or ~1 us of work), back to back.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

__global__ void empty_k(int* p) {
    if (p && threadIdx.x == 1023) p[0] = 1;
}
__global__ void work_k(float* p, int iters) {
    float a = threadIdx.x;
    for (int i = 0; i < iters; ++i) a = a * 1.0001f + 0.5f;
    if (a == -1.0f) p[0] = a;
}
__global__ void store_k(int4* out, long n) {
    long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
    long stride = (long)gridDim.x * blockDim.x;
    for (; i < n; i += stride) out[i] = make_int4((int)i, 1, 2, 255);
}

int main() {
    const long n = 4096L * 4096;
    int4* out;
    hipMalloc(&out, n * sizeof(int4));
    hipStream_t s;
    hipStreamCreate(&s);
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    auto run = [&](int mode, int reps) {
        for (int r = 0; r < reps; ++r) {
            if (mode >= 1) empty_k<<<16, 64, 0, s>>>(nullptr);
            if (mode >= 2) empty_k<<<4096, 64, 0, s>>>(nullptr);
            if (mode == 3) { work_k<<<16, 64, 0, s>>>(nullptr, 2000); }
            if (mode >= 0) store_k<<<65536, 256, 0, s>>>(out, n);
            if (mode == -1) empty_k<<<16, 64, 0, s>>>(nullptr);
        }
    };
    const char* names[] = {"store only", "empty(16) + store", "empty(16) + empty(4096) + store",
                           "empty(16) + empty(4096) + work(16,~2us) + store"};
    for (int round = 0; round < 3; ++round) {
        for (int mode = -1; mode < 4; ++mode) {
            run(mode, 20);
            hipStreamSynchronize(s);
            const int reps = 200;
            hipEventRecord(a, s);
            run(mode, reps);
            hipEventRecord(b, s);
            hipEventSynchronize(b);
            float ms;
            hipEventElapsedTime(&ms, a, b);
            std::printf("%-50s %7.2f us/iter\n", mode < 0 ? "empty(16) only" : names[mode],
                        ms * 1e3 / reps);
        }
    }
    return 0;
}
