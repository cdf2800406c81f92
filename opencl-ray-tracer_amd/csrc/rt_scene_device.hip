// rt_scene_device.hip -- the scene build on the device.
//
// The reference builds cubes on the host: Cube::Cube puts the 36 corners of
// the unit cube's 12 triangles into `triangles` (Cube.cpp:6-45), and
// Cube::scale / rotate / translate (Cube.cpp:53-83) each build one glm mat4
// and multiply every vertex by it, in call order.  createScene3
// (MainState.cpp:596-639) draws the transforms at random.  This file runs
// the same float arithmetic on the GPU, one lane per vertex, so a scene can
// be built (or re-transformed for animation) where it is rendered, with no
// host build and no upload.  The host restatement it must equal bit for bit
// is csrc/rt_scene.cpp (pinned against the reference's own Cube.cpp,
// oracle/ref_cube_shim.cpp).
//
// glm::rotate takes cos/sin of a float angle, i.e. glibc's cosf/sinf
// (matrix_transform.inl:52-58 -> std::cos(float)).  Those are not correctly
// rounded, so no device libm matches them.  glibc_sinf / glibc_cosf below
// restate glibc 2.35's algorithm (sysdeps/ieee754/flt-32/s_sinf.c, s_cosf.c,
// sincosf.h, sincosf_data.c: double-precision polynomial after a Cody-Waite
// or Payne-Hanek style reduction) as x86-64 glibc runs it on an FMA-capable
// CPU, the ifunc variants __sinf_fma / __cosf_fma, whose a * b + c steps are
// contracted to fused multiply-adds.  They equal the host's sinf / cosf on
// every finite float (scripts/check_glibc_sincosf.c, exhaustive).
//
// Build: -ffp-contract=off; the only fused operations are the explicit
// fma() calls of the restatement.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdint>
#include <cstring>

#include "rt_hip.h"
#include "rt_hip_debug.h"
#include "rt_internal.h"

#pragma clang fp contract(off)

namespace {

// ---- glibc 2.35 sinf / cosf, FMA variant ---------------------------------

// sincosf_data.c: __sincosf_table[0]; table [1] has c0..c4 negated.
constexpr double kHpiInv = 0x1.45F306DC9C883p+23;  // 2/pi * 2^24
constexpr double kHpi = 0x1.921FB54442D18p0;        // pi/2
constexpr double kC0 = 0x1p0, kC1 = -0x1.ffffffd0c621cp-2, kC2 = 0x1.55553e1068f19p-5,
                 kC3 = -0x1.6c087e89a359dp-10, kC4 = 0x1.99343027bf8c3p-16;
constexpr double kS1 = -0x1.555545995a603p-3, kS2 = 0x1.1107605230bc4p-7,
                 kS3 = -0x1.994eb3774cf24p-13;
constexpr double kPi63 = 0x1.921FB54442D18p-62;  // pi/2 * 2^-62
// 2/pi = 0x0.a2f9836e 4e441529 fc2757d1 f534ddc0 db629599 3c439041 ...
constexpr uint64_t kTwoOverPi[3] = {0xa2f9836e4e441529ull, 0xfc2757d1f534ddc0ull,
                                    0xdb6295993c439041ull};

__host__ __device__ inline uint32_t as_u32(float f) {
    uint32_t u;
    memcpy(&u, &f, sizeof u);
    return u;
}
// sincosf.h abstop12: the top 12 bits without the sign
__host__ __device__ inline uint32_t abstop12(float x) { return (as_u32(x) >> 20) & 0x7ff; }

// __inv_pio4[i] (sincosf_data.c): the 32 bits of 2/pi ending at byte i
__host__ __device__ inline uint32_t inv_pio4(int i) {
    uint32_t w = 0;
    for (int j = i - 3; j <= i; ++j) {
        const uint32_t b =
            j < 0 ? 0u : (uint32_t)(kTwoOverPi[j / 8] >> (56 - 8 * (j % 8))) & 0xffu;
        w = (w << 8) | b;
    }
    return w;
}

// sincosf.h sinf_poly; `neg` selects table [1]
__host__ __device__ inline float sinf_poly(double x, double x2, bool neg, int n) {
    if ((n & 1) == 0) {
        const double x3 = x * x2;
        const double s1 = fma(x2, kS3, kS2);
        const double x7 = x3 * x2;
        const double s = fma(x3, kS1, x);
        return (float)fma(x7, s1, s);
    }
    const double g = neg ? -1.0 : 1.0;  // exact: table [1] is table [0] with c negated
    const double x4 = x2 * x2;
    const double c2 = fma(x2, g * kC4, g * kC3);
    const double c1 = fma(x2, g * kC1, g * kC0);
    const double x6 = x4 * x2;
    const double c = fma(x4, g * kC2, c1);
    return (float)fma(x6, c2, c);
}

// sincosf.h reduce_fast (|x| < 120): x - n * pi/2
__host__ __device__ inline double reduce_fast(double x, int* np) {
    const double r = x * kHpiInv;
    const int n = ((int32_t)r + 0x800000) >> 24;
    *np = n;
    return fma(-(double)n, kHpi, x);
}

// sincosf.h reduce_large (|x| >= 120): 2/pi * x in 62-bit fixed point
__host__ __device__ inline double reduce_large(uint32_t xi, int* np) {
    const int a = (int)((xi >> 26) & 15);
    const int shift = (int)((xi >> 23) & 7);
    xi = (xi & 0xffffff) | 0x800000;
    xi <<= shift;
    uint64_t res0 = (uint64_t)(uint32_t)(xi * inv_pio4(a));
    const uint64_t res1 = (uint64_t)xi * inv_pio4(a + 4);
    const uint64_t res2 = (uint64_t)xi * inv_pio4(a + 8);
    res0 = (res2 >> 32) | (res0 << 32);
    res0 += res1;
    const uint64_t n = (res0 + (1ull << 61)) >> 62;
    res0 -= n << 62;
    *np = (int)n;
    return (double)(int64_t)res0 * kPi63;
}

constexpr uint32_t kTopPio4 = 0x3f4;   // abstop12(0x1.921FB6p-1f)
constexpr uint32_t kTopTiny = 0x398;   // abstop12(0x1p-12f)
constexpr uint32_t kTop120 = 0x42f;    // abstop12(120.0f)
constexpr uint32_t kTopInf = 0x7f8;    // abstop12(INFINITY)

// s_sinf.c
__host__ __device__ inline float glibc_sinf(float y) {
    double x = y;
    int n;
    const uint32_t t = abstop12(y);
    if (t < kTopPio4) {
        if (t < kTopTiny) return y;
        return sinf_poly(x, x * x, false, 0);
    }
    if (t < kTop120) {
        x = reduce_fast(x, &n);
        const double s = ((n & 3) == 1 || (n & 3) == 2) ? -1.0 : 1.0;  // sign[n & 3]
        return sinf_poly(x * s, x * x, (n & 2) != 0, n);
    }
    if (t < kTopInf) {
        const uint32_t xi = as_u32(y);
        const int sign = (int)(xi >> 31);
        x = reduce_large(xi, &n);
        const int m = n + sign;
        const double s = ((m & 3) == 1 || (m & 3) == 2) ? -1.0 : 1.0;
        return sinf_poly(x * s, x * x, (m & 2) != 0, n);
    }
    return (y - y) / (y - y);  // __math_invalidf: NaN for inf / NaN
}

// s_cosf.c
__host__ __device__ inline float glibc_cosf(float y) {
    double x = y;
    int n;
    const uint32_t t = abstop12(y);
    if (t < kTopPio4) {
        if (t < kTopTiny) return 1.0f;
        return sinf_poly(x, x * x, false, 1);
    }
    if (t < kTop120) {
        x = reduce_fast(x, &n);
        const double s = ((n & 3) == 1 || (n & 3) == 2) ? -1.0 : 1.0;
        return sinf_poly(x * s, x * x, (n & 2) != 0, n ^ 1);
    }
    if (t < kTopInf) {
        const uint32_t xi = as_u32(y);
        const int sign = (int)(xi >> 31);
        x = reduce_large(xi, &n);
        const int m = n + sign;
        const double s = ((m & 3) == 1 || (m & 3) == 2) ? -1.0 : 1.0;
        return sinf_poly(x * s, x * x, (m & 2) != 0, n ^ 1);
    }
    return (y - y) / (y - y);
}

// ---- Cube transforms (Cube.cpp:53-83 through glm 0.9.6.1) ------------------
// The same operation sequences as csrc/rt_scene.cpp, which the oracle pins
// against the reference's own Cube.cpp.

// Column-major 4x4, col[c][r], as glm::tmat4x4.
struct Mat4 {
    float col[4][4];
};

__device__ inline Mat4 mat_identity() {
    Mat4 m;
    for (int c = 0; c < 4; ++c)
        for (int r = 0; r < 4; ++r) m.col[c][r] = c == r ? 1.0f : 0.0f;
    return m;
}

// glm type_mat4x4.inl:596-607 -- (m0*v0 + m1*v1) + (m2*v2 + m3*v3)
__device__ inline float4 mat_apply(const Mat4& m, float4 v) {
    const float in[4] = {v.x, v.y, v.z, v.w};
    float r[4];
    for (int i = 0; i < 4; ++i) {
        const float lo = m.col[0][i] * in[0] + m.col[1][i] * in[1];
        const float hi = m.col[2][i] * in[2] + m.col[3][i] * in[3];
        r[i] = lo + hi;
    }
    return make_float4(r[0], r[1], r[2], r[3]);
}

// glm matrix_transform.inl:52-85 (radians), normalize = v * (1 / sqrt(dot(v, v)))
__device__ inline Mat4 mat_rotate(const Mat4& m, float angle, float ax, float ay, float az) {
    const float c = glibc_cosf(angle);
    const float s = glibc_sinf(angle);
    const float len2 = ax * ax + ay * ay + az * az;
    const float inv_len = 1.0f / sqrtf(len2);
    const float a[3] = {ax * inv_len, ay * inv_len, az * inv_len};
    const float k = 1.0f - c;
    const float t[3] = {k * a[0], k * a[1], k * a[2]};
    float rot[3][3];
    rot[0][0] = c + t[0] * a[0];
    rot[0][1] = 0.0f + t[0] * a[1] + s * a[2];
    rot[0][2] = 0.0f + t[0] * a[2] - s * a[1];
    rot[1][0] = 0.0f + t[1] * a[0] - s * a[2];
    rot[1][1] = c + t[1] * a[1];
    rot[1][2] = 0.0f + t[1] * a[2] + s * a[0];
    rot[2][0] = 0.0f + t[2] * a[0] + s * a[1];
    rot[2][1] = 0.0f + t[2] * a[1] - s * a[0];
    rot[2][2] = c + t[2] * a[2];
    Mat4 out;
    for (int j = 0; j < 3; ++j)
        for (int r = 0; r < 4; ++r)
            out.col[j][r] =
                m.col[0][r] * rot[j][0] + m.col[1][r] * rot[j][1] + m.col[2][r] * rot[j][2];
    for (int r = 0; r < 4; ++r) out.col[3][r] = m.col[3][r];
    return out;
}

// Cube::scale, Cube.cpp:65-73 (glm::scale, matrix_transform.inl:122-134)
__device__ inline float4 cube_scale(float4 v, float sx, float sy, float sz) {
    const Mat4 id = mat_identity();
    const float f[3] = {sx, sy, sz};
    Mat4 m;
    for (int j = 0; j < 3; ++j)
        for (int r = 0; r < 4; ++r) m.col[j][r] = id.col[j][r] * f[j];
    for (int r = 0; r < 4; ++r) m.col[3][r] = id.col[3][r];
    return mat_apply(m, v);
}

// Cube::rotate, Cube.cpp:53-63: rotate(rotate(rotate(I, z, Z), y, Y), x, X)
__device__ inline float4 cube_rotate(float4 v, float rx, float ry, float rz) {
    Mat4 m = mat_rotate(mat_identity(), rz, 0.0f, 0.0f, 1.0f);
    m = mat_rotate(m, ry, 0.0f, 1.0f, 0.0f);
    m = mat_rotate(m, rx, 1.0f, 0.0f, 0.0f);
    return mat_apply(m, v);
}

// Cube::translate, Cube.cpp:75-83 (glm::translate, matrix_transform.inl:40-50)
__device__ inline float4 cube_translate(float4 v, float tx, float ty, float tz) {
    Mat4 m = mat_identity();
    for (int r = 0; r < 4; ++r)
        m.col[3][r] = ((m.col[0][r] * tx + m.col[1][r] * ty) + m.col[2][r] * tz) + m.col[3][r];
    return mat_apply(m, v);
}

// Cube::Cube, Cube.cpp:10-45: corner k of the 12 triangles (bit0 = x,
// bit1 = y, bit2 = z; set bit = +1), the table of rt_scene.cpp.
__device__ inline float4 cube_corner(int k) {
    const unsigned char kCorners[36] = {0, 4, 6, 3, 0, 2, 5, 0, 1, 3, 1, 0, 0, 6, 2, 5, 4, 0,
                                        6, 4, 5, 7, 1, 3, 1, 7, 5, 7, 3, 2, 7, 2, 6, 7, 6, 5};
    const unsigned c = kCorners[k];
    return make_float4((c & 1u) ? 1.0f : -1.0f, (c & 2u) ? 1.0f : -1.0f,
                       (c & 4u) ? 1.0f : -1.0f, 1.0f);
}

// Utility::convertAngleToRadian, Utility.cpp:343-347
__device__ inline float deg_to_rad(float degrees) {
    const float pi = 3.1415926535f;
    return degrees * pi / 180.0f;
}

// One lane per vertex: vertex k of cube c, from the unit cube (or `in`),
// through the cube's ops in call order.
__global__ void __launch_bounds__(256) cube_build_kernel(const rt_cube_op* __restrict__ ops,
                                                        const int32_t* __restrict__ offsets,
                                                        int n_cubes, const float4* in,
                                                        float4* out) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= 36 * (int64_t)n_cubes) return;
    const int c = (int)(i / 36);
    float4 v = in ? in[i] : cube_corner((int)(i % 36));
    const int e = offsets[c + 1];
    for (int o = offsets[c]; o < e; ++o) {
        const rt_cube_op op = ops[o];
        if (op.op == RT_CUBE_SCALE)
            v = cube_scale(v, op.x, op.y, op.z);
        else if (op.op == RT_CUBE_ROTATE)
            v = cube_rotate(v, op.x, op.y, op.z);
        else if (op.op == RT_CUBE_TRANSLATE)
            v = cube_translate(v, op.x, op.y, op.z);
    }
    out[i] = v;
}

// ---- Synthetic scene (rt_scene_synthetic) -------------------
// The host draws one splitmix64 stream in order: 7 values per sphere, then
// 10 per cube.  Draw n's state is seed + (n + 1) * gamma, so every lane
// computes its own draws directly.
constexpr uint64_t kGamma = 0x9E3779B97F4A7C15ull;

__device__ inline float splitmix_uniform(uint64_t seed, int64_t n, float lo, float hi) {
    uint64_t z = seed + (uint64_t)(n + 1) * kGamma;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    z ^= z >> 31;
    const float unit = (float)(z >> 40) * (1.0f / 16777216.0f);
    return lo + unit * (hi - lo);
}

// Lanes [0, ns): spheres; then 36 lanes per cube (one per vertex; lane 0 of
// a cube also writes its colour).
__global__ void __launch_bounds__(256) synthetic_scene_kernel(
    float w, float h, int ns, int nc, uint64_t seed, float k, float4* __restrict__ so,
    float* __restrict__ sr, float4* __restrict__ sc, float4* __restrict__ cv,
    float4* __restrict__ cc) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < ns) {
        const int64_t d = 7 * i;
        const float x = splitmix_uniform(seed, d + 0, 0.0f, w);
        const float y = splitmix_uniform(seed, d + 1, 0.0f, h);
        const float z = -splitmix_uniform(seed, d + 2, 20.0f, 100.0f);
        so[i] = make_float4(x, y, z, 1.0f);
        sr[i] = splitmix_uniform(seed, d + 3, 5.0f, 30.0f) * k;
        sc[i] = make_float4(splitmix_uniform(seed, d + 4, 0.05f, 1.0f),
                            splitmix_uniform(seed, d + 5, 0.05f, 1.0f),
                            splitmix_uniform(seed, d + 6, 0.05f, 1.0f), 255.0f);
        return;
    }
    const int64_t j = i - ns;
    if (j >= 36 * (int64_t)nc) return;
    const int64_t c = j / 36;
    const int64_t d = 7 * (int64_t)ns + 10 * c;
    if (j % 36 == 0)
        cc[c] = make_float4(splitmix_uniform(seed, d + 0, 0.05f, 1.0f),
                            splitmix_uniform(seed, d + 1, 0.05f, 1.0f),
                            splitmix_uniform(seed, d + 2, 0.05f, 1.0f), 255.0f);
    const float s = splitmix_uniform(seed, d + 3, 5.0f, 30.0f) * k;
    const float az = splitmix_uniform(seed, d + 4, 0.0f, 359.0f);
    const float ay = splitmix_uniform(seed, d + 5, 0.0f, 359.0f);
    const float ax = splitmix_uniform(seed, d + 6, 0.0f, 359.0f);
    const float tx = splitmix_uniform(seed, d + 7, 0.0f, w);
    const float ty = splitmix_uniform(seed, d + 8, 0.0f, h);
    const float tz = -splitmix_uniform(seed, d + 9, 30.0f, 100.0f);
    float4 v = cube_corner((int)(j % 36));
    v = cube_scale(v, s, s, s);
    v = cube_rotate(v, 0.0f, 0.0f, deg_to_rad(az));
    v = cube_rotate(v, 0.0f, deg_to_rad(ay), 0.0f);
    v = cube_rotate(v, deg_to_rad(ax), 0.0f, 0.0f);
    v = cube_translate(v, tx, ty, tz);
    cv[j] = v;
}

// The restated sinf / cosf on the device, for the GPU test against the host
__global__ void sincosf_selftest_kernel(const float* in, int64_t n, float* s, float* c) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    s[i] = glibc_sinf(in[i]);
    c[i] = glibc_cosf(in[i]);
}

}  // namespace

namespace rt_internal {
// rt_init: load this translation unit's code object now (see preload() in
// rt_trace.inc)
int preload_scene_kernels() {
    hipFuncAttributes a;
    for (const void* k : {reinterpret_cast<const void*>(cube_build_kernel),
                          reinterpret_cast<const void*>(synthetic_scene_kernel)})
        if (hipFuncGetAttributes(&a, k) != hipSuccess) return RT_ERR_HIP;
    return RT_OK;
}
}  // namespace rt_internal

extern "C" {

int rt_cube_build_device(rt_ctx* ctx, const rt_cube_op* device_ops,
                         const int32_t* device_op_offsets, int32_t num_cubes,
                         const float* device_vertices_in, float* device_vertices_out,
                         void* stream) {
    if (!ctx || num_cubes < 0 || num_cubes > (1 << 24)) return RT_ERR_INVALID_ARG;
    if (num_cubes == 0) return RT_OK;
    if (!device_op_offsets || !device_vertices_out) return RT_ERR_INVALID_ARG;
    if (hipSetDevice(rt_internal::ctx_device(ctx)) != hipSuccess) return RT_ERR_HIP;
    hipStream_t st = stream ? static_cast<hipStream_t>(stream) : rt_internal::ctx_stream(ctx);
    if (!st) return RT_ERR_HIP;
    const int64_t n = 36 * (int64_t)num_cubes;
    cube_build_kernel<<<dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st>>>(
        device_ops, device_op_offsets, num_cubes,
        reinterpret_cast<const float4*>(device_vertices_in),
        reinterpret_cast<float4*>(device_vertices_out));
    return hipGetLastError() == hipSuccess ? RT_OK : RT_ERR_HIP;
}

int rt_scene_synthetic_device(rt_ctx* ctx, int32_t width, int32_t height, int32_t num_spheres,
                              int32_t num_cubes, uint64_t seed, float k, float* sphere_origins,
                              float* sphere_radius, float* sphere_colours, float* cube_vertices,
                              float* cube_colours, void* stream) {
    if (!ctx || width <= 0 || height <= 0 || num_spheres < 0 || num_cubes < 0 ||
        num_spheres > (1 << 28) || num_cubes > (1 << 24))
        return RT_ERR_INVALID_ARG;
    if ((num_spheres && (!sphere_origins || !sphere_radius || !sphere_colours)) ||
        (num_cubes && (!cube_vertices || !cube_colours)))
        return RT_ERR_INVALID_ARG;
    const int64_t n = num_spheres + 36 * (int64_t)num_cubes;
    if (n == 0) return RT_OK;
    if (hipSetDevice(rt_internal::ctx_device(ctx)) != hipSuccess) return RT_ERR_HIP;
    hipStream_t st = stream ? static_cast<hipStream_t>(stream) : rt_internal::ctx_stream(ctx);
    if (!st) return RT_ERR_HIP;
    synthetic_scene_kernel<<<dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st>>>(
        static_cast<float>(width), static_cast<float>(height), num_spheres, num_cubes, seed, k,
        reinterpret_cast<float4*>(sphere_origins), sphere_radius,
        reinterpret_cast<float4*>(sphere_colours), reinterpret_cast<float4*>(cube_vertices),
        reinterpret_cast<float4*>(cube_colours));
    return hipGetLastError() == hipSuccess ? RT_OK : RT_ERR_HIP;
}

int rt_selftest_sincosf(rt_ctx* ctx, const float* device_in, int64_t n, float* device_sin,
                        float* device_cos) {
    if (!ctx || n < 0 || (n && (!device_in || !device_sin || !device_cos)))
        return RT_ERR_INVALID_ARG;
    if (n == 0) return RT_OK;
    if (hipSetDevice(rt_internal::ctx_device(ctx)) != hipSuccess) return RT_ERR_HIP;
    hipStream_t st = rt_internal::ctx_stream(ctx);
    if (!st) return RT_ERR_HIP;
    sincosf_selftest_kernel<<<dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st>>>(
        device_in, n, device_sin, device_cos);
    if (hipGetLastError() != hipSuccess) return RT_ERR_HIP;
    return hipStreamSynchronize(st) == hipSuccess ? RT_OK : RT_ERR_HIP;
}

int rt_debug_glibc_sincosf(const float* x, int64_t n, float* sin_out, float* cos_out) {
    if (!x || n < 0 || !sin_out || !cos_out) return RT_ERR_INVALID_ARG;
    for (int64_t i = 0; i < n; ++i) {
        sin_out[i] = glibc_sinf(x[i]);
        cos_out[i] = glibc_cosf(x[i]);
    }
    return RT_OK;
}

}  // extern "C"
