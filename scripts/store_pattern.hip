// Store-pattern microbenchmark (large frames): one wave writes
// 4 KB of int32x4 pixels of a W x H frame (16 B per pixel) as
//   mode 0: 4 KB contiguous (4 rows of the same 1 KB-wide stripe order as a
//           linear fill: wave w writes bytes [4096 w, 4096 w + 4096));
//   mode 1: a 64 x 4 tile (four 1 KB row segments, W * 16 B apart), tiles in
//           the trace's order (16 tiles of a 64 x 64 bin, then bins row-major);
//   mode 2: a 256 x 1 tile (one 4 KB row segment), 64 x 16 tiles... in the
//           same bin order (4 tiles across, 16 down... see below);
//   mode 3: a 16 x 16 tile (sixteen 256 B segments), the 16 x 16 build's order;
//   mode 4: 64 x 4 tiles in frame-row-major tile order (consecutive waves
//           write adjacent 1 KB segments of the same four rows);
//   mode 5: 16 x 16 tiles in frame-row-major tile order;
//   mode 6: 4-wave workgroups, each wave a 64 x 4 tile of one of 4 adjacent
//           bins; the pixels go through LDS so that each wave stores one
//           whole 256-px row (4 KB contiguous), after a workgroup barrier.
// Built and run by hand: hipcc --offload-arch=gfx950 -O3 -o store_pattern
// store_pattern.hip && ./store_pattern 16384 16384
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

typedef int int4v __attribute__((ext_vector_type(4)));

template <int kMode>
__global__ void __launch_bounds__(64) store_kernel(int4v* out, int width, int n_bx) {
    const int lane = threadIdx.x;
    const long long w = blockIdx.x;
    const int4v v = {(int)w, lane, 7, 255};
    if (kMode == 0) {
        int4v* p = out + w * 256;
#pragma unroll
        for (int j = 0; j < 4; ++j) p[j * 64 + lane] = v;
    } else {
        // bins of 64 x 64 pixels, row-major; 16 waves per bin
        const long long bin = w / 16;
        const int t = (int)(w % 16);
        const long long bx = bin % n_bx, by = bin / n_bx;
        long long x0 = bx * 64, y0 = by * 64;
        if (kMode == 1) {  // 64 x 4 tiles stacked down the bin
            y0 += 4 * t;
#pragma unroll
            for (int j = 0; j < 4; ++j) out[(y0 + j) * width + x0 + lane] = v;
        } else if (kMode == 2) {  // 256 x 1 segments: the bin pair... 4 bins wide
            // 16 waves cover a 256 x 16 block: wave t writes row t, 4 KB
            const long long bx4 = bin % (n_bx / 4), by4 = bin / (n_bx / 4);
            const long long xs = bx4 * 256, ys = by4 * 16 + t;
#pragma unroll
            for (int j = 0; j < 4; ++j) out[ys * width + xs + j * 64 + lane] = v;
        } else if (kMode == 7) {
            const long long bx4 = bin % (n_bx / 4), by4 = bin / (n_bx / 4);
            const long long xs = bx4 * 256 + 128 * (t % 2), ys = by4 * 16 + 2 * (t / 2);
#pragma unroll
            for (int j = 0; j < 4; ++j) out[(ys + j / 2) * width + xs + (j % 2) * 64 + lane] = v;
        } else if (kMode == 8) {
            const long long n_by = (long long)gridDim.x / 16 / n_bx;
            const long long cx = bin / n_by, cy = bin % n_by;
            const long long xs = cx * 64, ys = cy * 64 + 4 * t;
#pragma unroll
            for (int j = 0; j < 4; ++j) out[(ys + j) * width + xs + lane] = v;
        } else if (kMode == 9) {
            const long long ys = y0 + (t / 4) + 16 * (t % 4);
#pragma unroll
            for (int j = 0; j < 4; ++j) out[(ys + 4 * j) * width + x0 + lane] = v;
        } else if (kMode == 10) {
            const long long bx4 = bin % (n_bx / 4), by4 = bin / (n_bx / 4);
            const long long xs = bx4 * 256 + 64 * (t % 4), ys = by4 * 16 + 4 * (t / 4);
#pragma unroll
            for (int j = 0; j < 4; ++j) out[(ys + j) * width + xs + lane] = v;
        } else if (kMode == 4) {
            const long long tx = w % n_bx, ty = w / n_bx;
#pragma unroll
            for (int j = 0; j < 4; ++j) out[(ty * 4 + j) * width + tx * 64 + lane] = v;
        } else if (kMode == 5) {
            const long long n_tx = width / 16, tx = w % n_tx, ty = w / n_tx;
#pragma unroll
            for (int j = 0; j < 4; ++j)
                out[(ty * 16 + 4 * j + lane / 16) * width + tx * 16 + lane % 16] = v;
        } else {  // 16 x 16 tiles, 4 x 4 per bin
            x0 += 16 * (t % 4);
            y0 += 16 * (t / 4);
#pragma unroll
            for (int j = 0; j < 4; ++j)
                out[(y0 + 4 * j + lane / 16) * width + x0 + lane % 16] = v;
        }
    }
}

__global__ void __launch_bounds__(256) store_exchange(int4v* out, int width, int n_bx) {
    __shared__ int4v s_pix[4][4][64];  // [row][wave][lane]
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const long long b = blockIdx.x;
    const long long g = b / 16;  // group of 4 bins along x
    const int t = (int)(b % 16);
    const long long bins_per_row = n_bx / 4;
    const long long gx = g % bins_per_row, gy = g / bins_per_row;
    const long long x0 = gx * 256, y0 = gy * 64 + 4 * t;
#pragma unroll
    for (int j = 0; j < 4; ++j) s_pix[j][wv][lane] = int4v{(int)b, lane, j, 255};
    __syncthreads();
#pragma unroll
    for (int k = 0; k < 4; ++k) out[(y0 + wv) * width + x0 + 64 * k + lane] = s_pix[wv][k][lane];
}

int main(int argc, char** argv) {
    const int width = argc > 1 ? atoi(argv[1]) : 16384;
    const int height = argc > 2 ? atoi(argv[2]) : 16384;
    const size_t n_px = (size_t)width * height;
    int4v* out = nullptr;
    if (hipMalloc(&out, n_px * 16) != hipSuccess) return 1;
    const unsigned waves = (unsigned)(n_px / 256);
    const int n_bx = width / 64;
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    const char* names[11] = {"linear 4 KB", "64x4 tiles", "256x1 rows", "16x16 tiles",
                            "64x4 rowmajor", "16x16 rowmaj", "64x4 via LDS", "128x2 tiles", "64x4 colmajor", "64x4 rows+4",
                             "64x4 256x16bin"};
    for (int rep = 0; rep < 3; ++rep) {
        for (int m = 0; m < 11; ++m) {
            auto launch = [&] {
                if (m == 0) store_kernel<0><<<waves, 64>>>(out, width, n_bx);
                if (m == 1) store_kernel<1><<<waves, 64>>>(out, width, n_bx);
                if (m == 2) store_kernel<2><<<waves, 64>>>(out, width, n_bx);
                if (m == 3) store_kernel<3><<<waves, 64>>>(out, width, n_bx);
                if (m == 4) store_kernel<4><<<waves, 64>>>(out, width, n_bx);
                if (m == 5) store_kernel<5><<<waves, 64>>>(out, width, n_bx);
                if (m == 6) store_exchange<<<waves / 4, 256>>>(out, width, n_bx);
                if (m == 7) store_kernel<7><<<waves, 64>>>(out, width, n_bx);
                if (m == 8) store_kernel<8><<<waves, 64>>>(out, width, n_bx);
                if (m == 9) store_kernel<9><<<waves, 64>>>(out, width, n_bx);
                if (m == 10) store_kernel<10><<<waves, 64>>>(out, width, n_bx);
            };
            launch();
            hipEventRecord(a);
            for (int i = 0; i < 10; ++i) launch();
            hipEventRecord(b);
            hipEventSynchronize(b);
            float ms = 0;
            hipEventElapsedTime(&ms, a, b);
            ms /= 10;
            printf("%dx%d %-12s %8.1f us  %.3f TB/s\n", width, height, names[m], ms * 1e3,
                   n_px * 16 / (ms * 1e-3) / 1e12);
        }
    }
    hipFree(out);
    return 0;
}
