// rt_device.hip -- MI355X (gfx950) ray-tracing kernels and the C ABI.
//
// Replaces the reference's OpenCL kernel rayTracer.cl::rayTracer
// (RayTrace/resources/shaders/rayTracer.cl:111-202) and its host dispatch
// MainState::executeRayTracerOpenCL (RayTrace/states/MainState.cpp:641-934).
// The numerics follow the reference's serial CPU path (MainState.cpp:257-408):
// fp64 Moller-Trumbore for cube triangles, fp32 glm sphere test, strict '<'
// closest hit in cubes-then-spheres order, depth-ramp shade, (int) stores.
//
// Three kernels per frame (DESIGN.md "Kernels"; scenes of at most 512
// primitives use two: prep, then trace_small_kernel, which bins its own tile):
//   prep   one lane per primitive: per-triangle fp64 constants, per-sphere
//          fp32 constants, and a conservative integer pixel box outside of
//          which the exact test provably rejects.
//   coarse one wave per 64x64 coarse bin: the ordered list of primitives
//          whose box touches the bin (ballot + mbcnt, the reference's
//          primitive order), each with a word of 2 bits per 16x16 wave tile
//          of the bin (tile classifier: skip / test / u,v proven inside).
//   trace  one wave per 16x16 tile, four pixels per lane (rows 4 apart):
//          count, ids, tile words and records all on scalar loads, exact
//          per-lane tests, 16-B coalesced framebuffer stores.
// Plus `generic`, a brute-force per-pixel kernel for arbitrary ray origins
// and directions (the reference's kernel arguments 8-9 in full generality).
//
// Build: -ffp-contract=off (and the pragma below): every operation rounds
// once, as x86-64 SSE does in the reference's CPU build.
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <thread>
#include <vector>

#include "rt_hip.h"
#include "rt_hip_debug.h"
#include "rt_internal.h"

#pragma clang fp contract(off)

namespace {

// Build-time geometry / feature knobs (A/B variants: scripts/variants.sh).
#ifndef RT_TILE_W
#define RT_TILE_W 16              // wave tile width (lanes per row); 8 (8x32 tiles) measured
                                  // 1.9 us per frame slower at config 3
#endif
#ifndef RT_ROWS
#define RT_ROWS 4                 // pixels per lane (rows, 64/RT_TILE_W apart)
#endif
#ifndef RT_TRACE_WAVES
#define RT_TRACE_WAVES 8          // amdgpu_waves_per_eu floor for trace (0 = none)
#endif
#ifndef RT_TIMELINE
#define RT_TIMELINE 0             // diagnostics: per-wave phase timestamps
#endif
constexpr int kWaveTile = RT_TILE_W;                       // wave tile width
constexpr int kRowsPerLane = RT_ROWS;
constexpr int kLaneRows = 64 / RT_TILE_W;                  // lane rows per pass
constexpr int kWaveTileH = kLaneRows * RT_ROWS;            // wave tile height
#ifndef RT_COARSE_W
#define RT_COARSE_W 64
#endif
#ifndef RT_COARSE_H
#define RT_COARSE_H 64
#endif
constexpr int kCoarseW = RT_COARSE_W;  // coarse bin (candidate list) size, pixels
constexpr int kCoarseH = RT_COARSE_H;
static_assert(kCoarseW % kWaveTile == 0 && kCoarseH % kWaveTileH == 0,
              "wave tiles must tile a coarse bin");
// prep_triangle's classifier margin covers tiles that overhang a box by up to
// kTileSpan pixels on any side
constexpr int kTileSpan = kWaveTile > kWaveTileH ? kWaveTile : kWaveTileH;
static_assert(kTileSpan <= 64, "tile span");
// Row blocks: the classifier's unit inside a wave tile.  Lane row j of a
// tile covers pixel rows tile_y + kLaneRows * j + [0, kLaneRows), i.e. one
// kWaveTile x kLaneRows block per j, so a per-block verdict (skip / test /
// u,v proven inside) is wave-uniform for each of a lane's rows.
// RT_ROWBITS 0 (default) classifies whole tiles (one block of kWaveTileH
// rows); 1 also classifies the row blocks of a triangle's partial tiles
// (measured slower: the trace saves 1.1 us, coarse pays 3.7 us).
#ifndef RT_ROWBITS
#define RT_ROWBITS 0
#endif
constexpr int kBlocks = RT_ROWBITS ? kRowsPerLane : 1;   // blocks per wave tile
constexpr int kBlockH = kWaveTileH / kBlocks;             // rows per block
constexpr int kTileBits = 2 * kBlocks;                    // bit 2b keep, 2b+1 inside
constexpr int kTilesPerWord = 32 / kTileBits;
constexpr unsigned kTileMask = kTileBits == 32 ? ~0u : (1u << kTileBits) - 1u;
constexpr unsigned kKeepMask = 0x55555555u & kTileMask;
static_assert(kBlockH * kBlocks == kWaveTileH && kTileBits <= 32, "row blocks");
// the block of lane row j
__host__ __device__ constexpr int row_block(int j) { return j * kBlocks / kRowsPerLane; }

constexpr int kThreads = 256;       // generic_kernel block
constexpr int kPrepThreads = 64;  // prep: one wave per block, spread over CUs
// Separable bin masks: a box overlaps a coarse bin iff it overlaps the bin's
// row of bins and its column of bins, so prep publishes, per bin row and per
// bin column, one 64-bit ballot per 64-primitive chunk, and a coarse wave
// ANDs its row's and column's words to get its candidates in primitive
// order without reading any box.  Frames with more than kMaskBinsMax bin
// rows + columns (extreme aspect ratios) scan the boxes instead.
constexpr int kMaskBinsMax = 4096;
#ifndef RT_BIN_MASKS
#define RT_BIN_MASKS 1            // default of rt_debug_set_bin_masks
#endif
constexpr double kEpsilon = 0.000001;      // MainState.cpp:15
constexpr float kFar = 300000.0f;          // MainState.cpp:345

typedef int int4v __attribute__((ext_vector_type(4)));

// Per-triangle constants of the binned path (128 B, scalar-loaded).
// With implicit origins (x, y, 0) and dir = (0, 0, D): pvec = d x e2 and
// det, inv_det are per-triangle; tvec = (x - v0x, y - v0y, -v0z) varies only
// in x and y.  Every field is produced by the same fp64 operation sequence as
// MainState.cpp:257-298, so per-pixel results are bit-identical.
struct alignas(16) TriRec {
    double v0x, v0y, p0, p1;
    double inv_det, e1x, e1y, e1z;
    double e2x, e2y, e2z, k0;  // k0 = tz * e1y
    double k1, dz, pad0, pad1; // k1 = tz * e1x, dz = D
};
static_assert(sizeof(TriRec) == 128, "TriRec layout");

// Per-sphere constants of the binned path (32 B).  With dir = (0, 0, D, Dw)
// and origins (x, y, 0, 1): tca = dot4(L, d) and the z/w half of dot4(L, L)
// do not depend on the pixel (MainState.cpp:300-327, glm pairwise dot).
// `fast` (1 or 0): every lane that can hit gets an r2 - dist2 in
// {0} u [2^-94, 2^102], where sqrt_rn_normal equals sqrtf (see prep_sphere).
// `tmin_key`: order_key of a lower bound of every lane's t0 (see prep_sphere;
// 0 = no bound), for depth culling in the trace.
struct alignas(16) SphRec {
    float cx, cy, kzw, tca2;  // kzw = Lz*Lz + Lw*Lw, tca2 = tca*tca
    float r2, tca, fast;
    unsigned tmin_key;
};
static_assert(sizeof(SphRec) == 32, "SphRec layout");

// Per-primitive tile classifier (32 B, fp32; evaluated by the coarse kernel).
// Triangle: a = (v0x, v0y, au, bu), b = (av, bv, g, 0) with the exact
// barycentrics u = au (x - v0x) + bu (y - v0y), v = av (x - v0x) + bv (y -
// v0y) up to a margin g that also covers the fp64 rounding of the per-pixel
// test, so a wave tile can be proven fully outside (skip) or fully inside
// (no u/v tests, t only) in fp32.  g = +inf disables both.
// Sphere: a = (cx, cy, R2, 0): every pixel farther than sqrt(R2) misses.
struct Cls {
    float4 a, b;
};
static_assert(sizeof(Cls) == 32, "Cls layout");

struct Box { int x0, y0, x1, y1; };  // inclusive pixel range, empty if x0 > x1

// Inverted far-out-of-range box: fails every overlap test against any pixel
// rectangle, so empty primitives can never reach a bin or a wave tile.
__host__ __device__ inline Box empty_box() {
    return Box{1 << 30, 1 << 30, -(1 << 30), -(1 << 30)};
}

// Unsigned key with the order of the float (for non-NaN values): positives
// above negatives, -0 just below +0.
__host__ __device__ inline unsigned order_key(float f) {
    unsigned b;
    memcpy(&b, &f, sizeof b);
    return b ^ ((b >> 31) ? 0xffffffffu : 0x80000000u);
}

__host__ __device__ inline bool finite3(double a, double b, double c) {
    return std::isfinite(a) && std::isfinite(b) && std::isfinite(c);
}

__host__ __device__ inline int clamp_floor(double v, int lo, int hi) {
    if (!(v > (double)lo)) return lo;
    if (!(v < (double)hi)) return hi;
    return (int)floor(v);
}
__host__ __device__ inline int clamp_ceil(double v, int lo, int hi) {
    if (!(v > (double)lo)) return lo;
    if (!(v < (double)hi)) return hi;
    return (int)ceil(v);
}

// Triangle prep.  Returns false when the triangle can never report a hit in
// the reference (|det| < EPSILON or a NaN det).  The box bound: outside the
// triangle's xy box by a distance Dist, the exact barycentric minimum is
// <= -Dist / (2 * extent); the computed u, v differ from the exact ones by
// at most `err` (rounding of e1, e2, pvec, det, tvec and the products), so
// a pad of 2 * extent * (2 * err + slack) (here x4 more) guarantees that
// the computed test rejects.  Ill-conditioned dets get the whole band.
__host__ __device__ inline bool prep_triangle(const float* a, const float* b, const float* c,
                                              double dx, double dy, double dz, int width,
                                              int row_begin, int row_end, TriRec* rec,
                                              Box* box, Cls* cls, bool* nonfinite) {
    const double v0[3] = {a[0], a[1], a[2]};
    const double v1[3] = {b[0], b[1], b[2]};
    const double v2[3] = {c[0], c[1], c[2]};
    *nonfinite = !(finite3(v0[0], v0[1], v0[2]) && finite3(v1[0], v1[1], v1[2]) &&
                   finite3(v2[0], v2[1], v2[2]));
    const double e1[3] = {v1[0] - v0[0], v1[1] - v0[1], v1[2] - v0[2]};
    const double e2[3] = {v2[0] - v0[0], v2[1] - v0[1], v2[2] - v0[2]};
    const double p0 = dy * e2[2] - dz * e2[1];
    const double p1 = dz * e2[0] - dx * e2[2];
    const double p2 = dx * e2[1] - dy * e2[0];
    const double det = e1[0] * p0 + e1[1] * p1 + e1[2] * p2;
    *box = empty_box();
    cls->a = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
    cls->b = make_float4(0.0f, 0.0f, INFINITY, 0.0f);
    if ((det > -kEpsilon && det < kEpsilon) || !(det == det) || *nonfinite) return false;
    const double inv_det = 1.0 / det;
    const double tz = 0.0 - v0[2];
    rec->v0x = v0[0];
    rec->v0y = v0[1];
    rec->p0 = p0;
    rec->p1 = p1;
    rec->inv_det = inv_det;
    rec->e1x = e1[0];
    rec->e1y = e1[1];
    rec->e1z = e1[2];
    rec->e2x = e2[0];
    rec->e2y = e2[1];
    rec->e2z = e2[2];
    rec->k0 = tz * e1[1];
    rec->k1 = tz * e1[0];
    rec->dz = dz;
    rec->pad0 = rec->pad1 = 0.0;

    const double eps = 1.1102230246251565e-16;  // 2^-53
    const double mnx = fmin(v0[0], fmin(v1[0], v2[0])), mxx = fmax(v0[0], fmax(v1[0], v2[0]));
    const double mny = fmin(v0[1], fmin(v1[1], v2[1])), mxy = fmax(v0[1], fmax(v1[1], v2[1]));
    // |tx|, |ty| bounds over the band, widened by one bin for tile overhang
    const double tx_max = fmax(fabs(0.0 - v0[0]), fabs((double)(width + 31) - v0[0])) + 1.0;
    const double ty_max =
        fmax(fabs((double)row_begin - v0[1]), fabs((double)(row_end + 31) - v0[1])) + 1.0;
    const double adet = fabs(det);
    const double rho =
        8.0 * eps * (fabs(e1[0] * p0) + fabs(e1[1] * p1) + fabs(e1[2] * p2)) / adet + 4.0 * eps;
    Box bx{0, row_begin, width - 1, row_end - 1};
    if (rho < 0.25) {
        const double s = (tx_max * (fabs(p0) + fabs(e1[1] * dz)) +
                          ty_max * (fabs(p1) + fabs(e1[0] * dz))) * fabs(inv_det);
        const double err = (32.0 * eps + 4.0 * rho) * s + 32.0 * eps;
        const double g = 2.0 * err + 8.0 * eps * s + 32.0 * eps;
        // fp32 classifier planes and their margin.  The classifier only ever
        // sees pixels of wave tiles (at most kTileSpan px on a side) that
        // overlap the box, so |x - v0x| and |y - v0y| are bounded by the padded
        // box plus kTileSpan: the margin
        // covers the fp64 test's rounding there (err_loc) and the fp32
        // rounding of the coefficients and of the plane evaluation (2^-24
        // each, x32 slack).
        const double padx0 = 8.0 * (mxx - mnx) * g + 0.5, pady0 = 8.0 * (mxy - mny) * g + 0.5;
        const double span = (double)kTileSpan;
        const double tx_loc = fmax(fabs(mnx - padx0 - span - v0[0]), fabs(mxx + padx0 + span - v0[0])) + 1.0;
        const double ty_loc = fmax(fabs(mny - pady0 - span - v0[1]), fabs(mxy + pady0 + span - v0[1])) + 1.0;
        const double s_loc = (tx_loc * (fabs(p0) + fabs(e1[1] * dz)) +
                              ty_loc * (fabs(p1) + fabs(e1[0] * dz))) * fabs(inv_det);
        const double err_loc = (32.0 * eps + 4.0 * rho) * s_loc + 32.0 * eps;
        const double g_loc = 2.0 * err_loc + 8.0 * eps * s_loc + 32.0 * eps;
        const double au = p0 * inv_det, bu = p1 * inv_det;
        const double av = dz * e1[1] * inv_det, bv = -(dz * e1[0]) * inv_det;
        const double suv = (fabs(au) + fabs(av)) * tx_loc + (fabs(bu) + fabs(bv)) * ty_loc;
        const double gm = g_loc + 32.0 * 5.9604644775390625e-08 * suv + 1e-6;
        cls->a = make_float4((float)v0[0], (float)v0[1], (float)au, (float)bu);
        cls->b = make_float4((float)av, (float)bv, (float)(gm * (1.0 + 1e-6)), 0.0f);
        const double padx = 8.0 * (mxx - mnx) * g + 0.5;
        const double pady = 8.0 * (mxy - mny) * g + 0.5;
        bx.x0 = clamp_floor(mnx - padx, 0, width - 1);
        bx.x1 = clamp_ceil(mxx + padx, 0, width - 1);
        bx.y0 = clamp_floor(mny - pady, row_begin, row_end - 1);
        bx.y1 = clamp_ceil(mxy + pady, row_begin, row_end - 1);
        // wholly outside the band / frame?
        if (mxx + padx < 0.0 || mnx - padx > (double)(width - 1) ||
            mxy + pady < (double)row_begin || mny - pady > (double)(row_end - 1))
            return true;  // box stays empty
    }
    *box = bx;
    return true;
}

// Sphere prep (fp32, MainState.cpp:300-327 with glm's pairwise vec4 dot).
// Miss is guaranteed where |L|^2 (1 - 8e) > r2 - (kzw - tca2) + 8e(|kzw| +
// |tca2|), e = 2^-23 (bound on the fp32 rounding of Lx, Ly, their squares
// and the two sums); the box is that radius plus one pixel.
__host__ __device__ inline void prep_sphere(const float* o, float radius, float dx, float dy,
                                            float dz, float dw, int width, int row_begin,
                                            int row_end, SphRec* rec, Box* box, Cls* cls,
                                            bool* nonfinite) {
    *box = empty_box();
    cls->a = make_float4(o[0], o[1], -1.0f, 0.0f);
    cls->b = make_float4(0.0f, 0.0f, 0.0f, 1.0f);
    *nonfinite = !(std::isfinite(o[0]) && std::isfinite(o[1]) && std::isfinite(o[2]) &&
                   std::isfinite(o[3]) && std::isfinite(radius));
    const float lz = o[2] - 0.0f;
    const float lw = o[3] - 1.0f;
    const float tca = (lz * dz) + (lw * dw);  // + (Lx*dx + Ly*dy) == +-0
    const float kzw = (lz * lz) + (lw * lw);
    const float tca2 = tca * tca;
    const float r2 = radius * radius;
    rec->cx = o[0];
    rec->cy = o[1];
    rec->kzw = kzw;
    rec->tca2 = tca2;
    rec->r2 = r2;
    rec->tca = tca;
    // r2 >= 2^-70: a hitting lane has dist2 <= r2, so r2 - dist2 is 0, or
    // >= r2 / 2 (dist2 <= r2 / 2), or an exact nonzero difference of floats
    // >= r2 / 2, a multiple of ulp(2^-71) = 2^-94.  The 2^100 caps keep
    // dist2 >= -2^101, so r2 - dist2 <= 2^102 (and tca2 finite).
    rec->fast = (r2 >= 0x1p-70f && r2 <= 0x1p100f && fabsf(tca2) <= 0x1p100f &&
                 fabsf(kzw) <= 0x1p100f) ? 1.0f : 0.0f;
    // Lower bound of t0 over all pixels, by monotonicity of IEEE rounding:
    // lx*lx + ly*ly >= 0, so dist2 = ((.) + kzw) - tca2 >= kzw - tca2 = d0,
    // arg = r2 - dist2 <= r2 - d0 = a0, thc <= sqrtf(a0) (correctly rounded
    // on both sides), t0 = tca - thc >= tca - sqrtf(a0).  The same float ops
    // in the same order, so the bound holds for the computed values.
    {
        const float d0 = kzw - tca2;
        const float a0 = r2 - d0;
        const float tmin = tca - sqrtf(a0);
        rec->tmin_key = tmin == tmin ? order_key(tmin) : 0u;  // NaN: no bound
    }
    (void)dx;
    (void)dy;
    if (*nonfinite || !(tca >= 0.0f)) return;  // tca < 0 (or NaN): never a hit
    const double e = 1.1920928955078125e-07;  // 2^-23
    const double bound = ((double)r2 - ((double)kzw - (double)tca2) +
                          8.0 * e * (fabs((double)kzw) + fabs((double)tca2))) /
                         (1.0 - 8.0 * e);
    if (!(bound >= 0.0)) return;  // every pixel misses
    const double r = sqrt(bound * (1.0 + 1e-6) + 1e-6) + 1.0;
    cls->a.z = (float)(bound * (1.0 + 1e-5) + 1e-5);
    const double cx = o[0], cy = o[1];
    if (cx + r < 0.0 || cx - r > (double)(width - 1) || cy + r < (double)row_begin ||
        cy - r > (double)(row_end - 1))
        return;
    box->x0 = clamp_floor(cx - r, 0, width - 1);
    box->x1 = clamp_ceil(cx + r, 0, width - 1);
    box->y0 = clamp_floor(cy - r, row_begin, row_end - 1);
    box->y1 = clamp_ceil(cy + r, row_begin, row_end - 1);
}

// (int)f as x86-64 cvttss2si: truncation, NaN / out of range -> INT32_MIN.
__device__ __forceinline__ int cvt_i32(float f) {
    return (f >= -2147483648.0f && f < 2147483648.0f) ? (int)f : INT32_MIN;
}

// The same on the hot path: v_cvt_i32_f32 truncates and saturates (-inf and
// everything below -2^31 -> INT32_MIN, NaN -> 0, >= 2^31 -> INT32_MAX); the
// one compare maps NaN and >= 2^31 to x86's INT32_MIN.  Inline asm keeps the
// hardware semantics (a C++ (int) of an out-of-range float is undefined).
__device__ __forceinline__ int cvt_i32_fast(float f) {
    int r;
    asm volatile("v_cvt_i32_f32 %0, %1" : "=v"(r) : "v"(f));
    return f < 2147483648.0f ? r : INT32_MIN;
}

// Correctly rounded x / 180.0f without the IEEE division sequence:
// q0 = x * RN(1/180), q = fma(fma(-q0, 180, x), RN(1/180), q0) equals RN(x/180)
// for every finite float with |x| >= 2^-100 (exhaustively checked on the host,
// scripts/check_div180.c); smaller |x| takes the division.
__device__ __forceinline__ float div180(float x) {
    const float r = 1.0f / 180.0f;
    const float q0 = x * r;
    const float rem = __builtin_fmaf(-q0, 180.0f, x);
    float q = __builtin_fmaf(rem, r, q0);
    const bool tiny = !(__builtin_fabsf(x) >= 0x1p-100f);
    if (__ballot(tiny)) q = tiny ? x / 180.0f : q;
    return q;
}

// MainState.cpp:396-407 + :952-955 (or the Texture packing :1026-1036).
__device__ __forceinline__ int4v shade(float closest, float4 colour) {
    if (closest == kFar) return int4v{0, 0, 0, 255};
    const float normalised = (closest - 0.0f) / (180.0f - 0.0f);
    const float scalar = 255.0f - (normalised * 255.0f);
    return int4v{cvt_i32(scalar * colour.x), cvt_i32(scalar * colour.y),
                 cvt_i32(scalar * colour.z), 255};
}

__device__ __forceinline__ unsigned pack_rgba8(int4v p) {
    return (unsigned)(unsigned char)p.x | ((unsigned)(unsigned char)p.y << 8) |
           ((unsigned)(unsigned char)p.z << 16) | 0xFF000000u;
}

// ---------------------------------------------------------------------------
// Generic per-pixel path: the reference algorithm verbatim (any origin and
// direction).  MainState.cpp:257-298 (fp64 MT), :300-327, :330-408.
// ---------------------------------------------------------------------------
__device__ inline int intersect_tri(const double* orig, const double* dir, const double* v0,
                                    const double* v1, const double* v2, double* t) {
    double e1[3], e2[3], tv[3], pv[3], qv[3];
    e1[0] = v1[0] - v0[0]; e1[1] = v1[1] - v0[1]; e1[2] = v1[2] - v0[2];
    e2[0] = v2[0] - v0[0]; e2[1] = v2[1] - v0[1]; e2[2] = v2[2] - v0[2];
    pv[0] = dir[1] * e2[2] - dir[2] * e2[1];
    pv[1] = dir[2] * e2[0] - dir[0] * e2[2];
    pv[2] = dir[0] * e2[1] - dir[1] * e2[0];
    const double det = e1[0] * pv[0] + e1[1] * pv[1] + e1[2] * pv[2];
    if (det > -kEpsilon && det < kEpsilon) return 0;
    const double inv_det = 1.0 / det;
    tv[0] = orig[0] - v0[0]; tv[1] = orig[1] - v0[1]; tv[2] = orig[2] - v0[2];
    const double u = (tv[0] * pv[0] + tv[1] * pv[1] + tv[2] * pv[2]) * inv_det;
    if (u < 0.0 || u > 1.0) return 0;
    qv[0] = tv[1] * e1[2] - tv[2] * e1[1];
    qv[1] = tv[2] * e1[0] - tv[0] * e1[2];
    qv[2] = tv[0] * e1[1] - tv[1] * e1[0];
    const double v = (dir[0] * qv[0] + dir[1] * qv[1] + dir[2] * qv[2]) * inv_det;
    if (v < 0.0 || u + v > 1.0) return 0;
    *t = (e2[0] * qv[0] + e2[1] * qv[1] + e2[2] * qv[2]) * inv_det;
    return 1;
}

__device__ inline float dot4(float4 a, float4 b) {
    return ((a.x * b.x) + (a.y * b.y)) + ((a.z * b.z) + (a.w * b.w));
}

__device__ inline float intersect_sphere(float4 o, float4 d, float radius, float4 c) {
    const float4 l = make_float4(c.x - o.x, c.y - o.y, c.z - o.z, c.w - o.w);
    const float tca = dot4(l, d);
    if (tca < 0) return 0.0f;
    const float dist2 = dot4(l, l) - tca * tca;
    const float r2 = radius * radius;
    if (dist2 > r2) return 0.0f;
    const float thc = sqrtf(r2 - dist2);
    return tca - thc;
}

struct SceneDev {
    const float4* __restrict__ sphere_origins;
    const float* __restrict__ sphere_radius;
    const float4* __restrict__ sphere_colours;
    const float4* __restrict__ cube_vertices;
    const float4* __restrict__ cube_colours;
    int n_spheres, n_cubes;
};

__device__ inline int4v collide_generic(const SceneDev& s, float4 origin, float4 dir) {
    const double o[3] = {origin.x, origin.y, origin.z};
    const double d[3] = {dir.x, dir.y, dir.z};
    float closest = kFar;
    float4 colour = make_float4(0.0f, 0.0f, 0.0f, 255.0f);
    for (int c = 0; c < s.n_cubes; ++c) {
        const float4* tri = s.cube_vertices + 36 * c;
        for (int k = 0; k < 36; k += 3) {
            const float4 a = tri[k], b = tri[k + 1], e = tri[k + 2];
            const double v0[3] = {a.x, a.y, a.z}, v1[3] = {b.x, b.y, b.z}, v2[3] = {e.x, e.y, e.z};
            double t;
            if (intersect_tri(o, d, v0, v1, v2, &t) == 1 && (float)t < closest) {
                closest = (float)t;
                colour = s.cube_colours[c];
            }
        }
    }
    for (int i = 0; i < s.n_spheres; ++i) {
        const float dist = intersect_sphere(origin, dir, s.sphere_radius[i], s.sphere_origins[i]);
        if (dist == 0.0f) continue;
        if (dist < closest) {
            closest = dist;
            colour = s.sphere_colours[i];
        }
    }
    return shade(closest, colour);
}

__global__ void __launch_bounds__(kThreads) generic_kernel(
    SceneDev scene, float4 dir, const float4* __restrict__ origins, int width,
    int row_begin, int row_end, int out_format, void* __restrict__ out) {
    // grid-stride: the AQL grid counts work-items in 32 bits, frames may not
    const int64_t n = (int64_t)width * (row_end - row_begin);
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        const int x = (int)(i % width);
        const int y = row_begin + (int)(i / width);
        // `origins` starts at row row_begin (the band's rows only)
        const float4 o = origins ? origins[i] : make_float4((float)x, (float)y, 0.0f, 1.0f);
        const int4v p = collide_generic(scene, o, dir);
        if (out_format == RT_FORMAT_I32X4)
            reinterpret_cast<int4v*>(out)[i] = p;
        else
            reinterpret_cast<unsigned*>(out)[i] = pack_rgba8(p);
    }
}

// ---------------------------------------------------------------------------
// Binned path
// ---------------------------------------------------------------------------
// Bin masks (`row_masks` != nullptr): after its records and boxes, each prep
// wave (one 64-primitive chunk) writes row_masks[r * n_chunks + chunk] and
// col_masks[c * n_chunks + chunk]: the ballot of its primitives whose box
// overlaps bin row r / bin column c.  Every word is written every frame.
__global__ void __launch_bounds__(kPrepThreads) prep_kernel(
    SceneDev scene, float4 dir, int width, int row_begin, int row_end,
    TriRec* __restrict__ tri, SphRec* __restrict__ sph, int4* __restrict__ boxes,
    Cls* __restrict__ cls, float4* __restrict__ colours, unsigned* __restrict__ nonfinite_flag,
    unsigned gen, unsigned long long* __restrict__ row_masks,
    unsigned long long* __restrict__ col_masks, int n_cx, int n_cy) {
    const int n_tri = 12 * scene.n_cubes;
    const int n_prims = n_tri + scene.n_spheres;
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    const int lane = threadIdx.x;
    Box b = empty_box();
    Cls k{};
    bool bad = false;
    if (i < n_tri) {
        const float4* v = scene.cube_vertices + 3 * i;
        const float4 a = v[0], bb = v[1], c = v[2];
        const float fa[3] = {a.x, a.y, a.z}, fb[3] = {bb.x, bb.y, bb.z}, fc[3] = {c.x, c.y, c.z};
        if (i % 12 == 0) colours[i / 12] = scene.cube_colours[i / 12];
        TriRec r{};
        prep_triangle(fa, fb, fc, (double)dir.x, (double)dir.y, (double)dir.z, width, row_begin,
                      row_end, &r, &b, &k, &bad);
        tri[i] = r;
    } else if (i < n_prims) {
        const int s = i - n_tri;
        const float4 o = scene.sphere_origins[s];
        colours[scene.n_cubes + s] = scene.sphere_colours[s];
        const float fo[4] = {o.x, o.y, o.z, o.w};
        SphRec r{};
        prep_sphere(fo, scene.sphere_radius[s], dir.x, dir.y, dir.z, dir.w, width, row_begin,
                    row_end, &r, &b, &k, &bad);
        sph[s] = r;
    }
    if (i < n_prims) {
        boxes[i] = make_int4(b.x0, b.y0, b.x1, b.y1);
        cls[i] = k;
        if (bad) atomicMax(nonfinite_flag, gen);
    }
    if (!row_masks) return;
    const int chunk = (int)blockIdx.x;
    const int n_chunks = (int)gridDim.x;
    const bool live = i < n_prims && b.x0 <= b.x1 && b.y0 <= b.y1;
    // Per block of 64 bins, lane r builds bin r's word without a ballot per
    // bin: first[r] / last[r] collect the primitives whose box starts / ends
    // in bin r (LDS OR), a prefix OR of first and a suffix OR of last (plus
    // the primitives starting before / ending after the block) give the
    // primitives with start <= r and end >= r; their AND is bin r's word.
    __shared__ unsigned long long s_first[64], s_last[64];
    auto bin_words = [&](int lo, int hi, int n_bins, int bin_px, unsigned long long* out) {
        const int blo = live ? lo / bin_px : INT32_MAX;
        const int bhi = live ? hi / bin_px : -1;
        const unsigned long long me = 1ull << lane;
        for (int r0 = 0; r0 < n_bins; r0 += 64) {
            s_first[lane] = 0ull;
            s_last[lane] = 0ull;
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            if (blo >= r0 && blo < r0 + 64) atomicOr(&s_first[blo - r0], me);
            if (bhi >= r0 && bhi < r0 + 64) atomicOr(&s_last[bhi - r0], me);
            __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
            __builtin_amdgcn_wave_barrier();
            unsigned long long f = s_first[lane], e = s_last[lane];
            const unsigned long long f_in = __ballot(blo < r0);        // started before
            const unsigned long long e_in = __ballot(bhi >= r0 + 64 && bhi != -1);  // ends after
#pragma unroll
            for (int off = 1; off < 64; off <<= 1) {
                const unsigned long long fu = __shfl_up(f, off);
                const unsigned long long ed = __shfl_down(e, off);
                if (lane >= off) f |= fu;
                if (lane + off < 64) e |= ed;
            }
            if (r0 + lane < n_bins)
                out[(int64_t)(r0 + lane) * n_chunks + chunk] = (f | f_in) & (e | e_in);
            __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
            __builtin_amdgcn_wave_barrier();
        }
    };
    bin_words(b.y0 - row_begin, b.y1 - row_begin, n_cy, kCoarseH, row_masks);
    bin_words(b.x0, b.x1, n_cx, kCoarseW, col_masks);
}

#if RT_TIMELINE
// per wave: realtime at entry / first staged / walked / stores issued,
// s_memtime at entry / end, HW_ID, XCC_ID
__device__ unsigned* g_timeline;
__device__ __forceinline__ unsigned rt_now() { return (unsigned)__builtin_amdgcn_s_memrealtime(); }
#define TL_MARK(v) const unsigned v = rt_now()
#else
#define TL_MARK(v)
#endif

// Per-lane exact tests of one candidate primitive `p` (wave-uniform) on the
// lane's kRowsPerLane pixels.  Triangles: MainState.cpp:257-298 restated on
// the per-triangle constants (see TriRec); `inside` (wave-uniform) means the
// tile classifier proved every pixel of the tile passes the u/v tests, so
// only the exact t is computed.  Spheres: :300-327 on SphRec.
// Select-based form: every row evaluates the whole test and a compare picks
// the result, so the wave never diverges inside the walk.  The per-lane
// (row-invariant) products are hoisted; each is the same fp64 operation on
// the same operands as in MainState.cpp:257-298, so values are unchanged.
#ifndef RT_ROWSKIP
#define RT_ROWSKIP 0  // 1: skip triangle rows, 2: sphere rows, 3: both (no lane can hit)
#endif
#ifndef RT_ROWSKIP_RGBA8
#define RT_ROWSKIP_RGBA8 0  // the same for the Texture (RGBA8) trace (1-3 measured slower)
#endif
// Row skipping per output format: the int32x4 trace hides its test VALU
// under the store drain (measured slower with skips), the RGBA8 trace is
// VALU-bound.
template <int kFmt>
constexpr int row_skip() { return kFmt == RT_FORMAT_RGBA8 ? RT_ROWSKIP_RGBA8 : RT_ROWSKIP; }

template <int kSkip = RT_ROWSKIP>
__device__ __forceinline__ void test_tri(const TriRec& r, int slot, unsigned bits, double px,
                                         const double* py, float* closest, int* hit) {
    const double tx = px - r.v0x;
    const double txe1y = tx * r.e1y;               // q2 = tx*e1y - ty*e1x
    const double q1 = r.k1 - tx * r.e1z;           // q1 = tz*e1x - tx*e1z
    const double e2yq1 = r.e2y * q1;
    const double txp0 = tx * r.p0;                 // u = (tx*p0 + ty*p1) * inv_det
#pragma unroll
    for (int j = 0; j < kRowsPerLane; ++j) {
        // this row's block: bit 0 keep, bit 1 u,v proven inside (wave-uniform)
        const unsigned rb = bits >> (2 * row_block(j));
        if (!(rb & 1u)) continue;
        const double ty = py[j] - r.v0y;
        const double q2 = txe1y - ty * r.e1x;
        bool pass = true;
        if (!(rb & 2u)) {
            const double u = (txp0 + ty * r.p1) * r.inv_det;
            const double v = (r.dz * q2) * r.inv_det;
            pass = !((u < 0.0) | (u > 1.0) | (v < 0.0) | (u + v > 1.0));
            // no lane of this row inside the triangle: its t is never used
            if ((kSkip & 1) && __ballot(pass) == 0ull) continue;
        }
        const double q0 = ty * r.e1z - r.k0;
        const double t = ((r.e2x * q0 + e2yq1) + r.e2z * q2) * r.inv_det;
        const float tf = (float)t;
        const bool take = pass & (tf < closest[j]);
        closest[j] = take ? tf : closest[j];
        hit[j] = take ? slot : hit[j];
    }
}

// Correctly rounded sqrtf for x in [2^-96, FLT_MAX]: v_sqrt_f32 plus the two
// FMA residual corrections of the compiler's IEEE expansion, without its
// denormal scaling and zero/inf fix-up (equal to sqrtf on every float of
// that range: exhaustive check, scripts/check_sqrt.hip).
__device__ __forceinline__ float sqrt_rn_normal(float x) {
    const float s = __builtin_amdgcn_sqrtf(x);
    const int si = __builtin_bit_cast(int, s);
    const float sm = __builtin_bit_cast(float, si - 1);
    const float sp = __builtin_bit_cast(float, si + 1);
    float r = __builtin_fmaf(-sm, s, x) <= 0.0f ? sm : s;
    r = __builtin_fmaf(-sp, s, x) > 0.0f ? sp : r;
    return r;
}

template <int kSkip = RT_ROWSKIP>
__device__ __forceinline__ void test_sph(const SphRec& s, int slot, unsigned bits, float pxf,
                                         const float* pyf, float* closest, int* hit) {
    const float lx = s.cx - pxf;
    const float lx2 = lx * lx;
    float dist2[kRowsPerLane], arg[kRowsPerLane];
#pragma unroll
    for (int j = 0; j < kRowsPerLane; ++j) {
        const float ly = s.cy - pyf[j];
        const float a = lx2 + ly * ly;
        dist2[j] = (a + s.kzw) - s.tca2;
        arg[j] = s.r2 - dist2[j];
    }
    // per sphere (scalar): the general sqrtf only where a hitting lane's
    // argument could leave the range sqrt_rn_normal is exact on
    const bool general = !(s.fast != 0.0f);
#pragma unroll
    for (int j = 0; j < kRowsPerLane; ++j) {
        if (!((bits >> (2 * row_block(j))) & 1u)) continue;  // block skipped (uniform)
        // no lane of this row within the sphere's disc: nothing to update
        if ((kSkip & 2) && __ballot(!(dist2[j] > s.r2)) == 0ull) continue;
        const float thc = general ? sqrtf(arg[j]) : sqrt_rn_normal(arg[j]);
        const float t0 = s.tca - thc;
        // dist2 > r2 (a miss, MainState.cpp:314) makes arg = r2 - dist2 < 0
        // (the sign of a difference of floats is exact), so thc and t0 are
        // NaN and `t0 < closest` fails: the miss test needs no compare of
        // its own.  A NaN dist2 gives a NaN t0 as well.
        const bool take = (t0 != 0.0f) & (t0 < closest[j]);
        closest[j] = take ? t0 : closest[j];
        hit[j] = take ? slot : hit[j];
    }
}

// Tile classification of one candidate against the rectangle
// [x0, x0+kW-1] x [y0, y0+kH-1] (fp32, conservative; see Cls).
template <int kWpx = kWaveTile, int kHpx = kWaveTileH>
__device__ __forceinline__ void classify(const Cls& k, bool is_tri, float x0, float y0,
                                         bool* keep, bool* inside) {
    constexpr float kW = (float)(kWpx - 1), kH = (float)(kHpx - 1);
    if (is_tri) {
        const float xl = x0 - k.a.x, xh = (x0 + kW) - k.a.x;
        const float yl = y0 - k.a.y, yh = (y0 + kH) - k.a.y;
        const float u1 = k.a.z * xl, u2 = k.a.z * xh, u3 = k.a.w * yl, u4 = k.a.w * yh;
        const float v1 = k.b.x * xl, v2 = k.b.x * xh, v3 = k.b.y * yl, v4 = k.b.y * yh;
        const float umin = fminf(u1, u2) + fminf(u3, u4), umax = fmaxf(u1, u2) + fmaxf(u3, u4);
        const float vmin = fminf(v1, v2) + fminf(v3, v4), vmax = fmaxf(v1, v2) + fmaxf(v3, v4);
        const float g = k.b.z;
        const bool out = umax < -g || umin > 1.0f + g || vmax < -g || vmin > 1.0f + g ||
                         umin + vmin > 1.0f + g;
        *keep = !out;
        *inside = umin > g && umax < 1.0f - g && vmin > g && vmax < 1.0f - g &&
                  umax + vmax < 1.0f - g;
    } else {
        const float dx = fmaxf(fmaxf(x0 - k.a.x, k.a.x - (x0 + kW)), 0.0f);
        const float dy = fmaxf(fmaxf(y0 - k.a.y, k.a.y - (y0 + kH)), 0.0f);
        *keep = !(dx * dx + dy * dy > k.a.z);
        *inside = false;
    }
}

// Pixel value of the Texture format (MainState.cpp:1026-1036) or int32x4.
template <int kFmt>
__device__ __forceinline__ void store_fmt(void* __restrict__ out, int64_t idx, int4v pix) {
    if (kFmt == RT_FORMAT_I32X4)
        reinterpret_cast<int4v*>(out)[idx] = pix;
    else
        reinterpret_cast<unsigned*>(out)[idx] = pack_rgba8(pix);
}

// The same for shade_pixels' output: RGBA8 words arrive packed in pix.x.
template <int kFmt>
__device__ __forceinline__ void store_shaded(void* __restrict__ out, int64_t idx, int4v pix) {
    if (kFmt == RT_FORMAT_I32X4)
        reinterpret_cast<int4v*>(out)[idx] = pix;
    else
        reinterpret_cast<unsigned*>(out)[idx] = (unsigned)pix.x;
}

// The Texture packing (MainState.cpp:1026-1036) of three (int) channels.
__device__ __forceinline__ unsigned pack_bytes(int r, int g, int b) {
    return ((unsigned)r & 0xffu) | (((unsigned)g & 0xffu) << 8) | (((unsigned)b & 0xffu) << 16) |
           0xFF000000u;
}

// Shade (MainState.cpp:396-407) one lane's kRowsPerLane pixels.  Int32x4:
// pix[j] is the pixel.  RGBA8: pix[j].x is the packed Texture word.
template <int kMode = 0, int kFmt = RT_FORMAT_I32X4>
__device__ __forceinline__ void shade_pixels(const float4* __restrict__ colours,
                                             const float* closest, const int* hit, int4v* pix) {
    bool lane_hit = false;
#pragma unroll
    for (int j = 0; j < kRowsPerLane; ++j) lane_hit |= hit[j] >= 0;
    const bool any_hit = __ballot(lane_hit) != 0ull;
    if (kFmt == RT_FORMAT_RGBA8) {
        // The Texture keeps the low byte of each (int) channel.  x86's (int)
        // gives INT32_MIN (low byte 0) for NaN, +-inf and |f| >= 2^31;
        // v_cvt_i32_f32 agrees on that byte except for f >= 2^31 (it
        // saturates to 0x7fffffff), so one wave-uniform max3 test replaces
        // the per-channel fix-ups of cvt_i32_fast on the common path.
#pragma unroll
        for (int j = 0; j < kRowsPerLane; ++j) pix[j].x = (int)0xFF000000u;
        if (!any_hit) return;
        float4 col[kRowsPerLane];
#pragma unroll
        for (int j = 0; j < kRowsPerLane; ++j)
            col[j] = kMode == 4 ? make_float4(1.0f, 0.5f, 0.25f, 255.0f)
                                : colours[hit[j] >= 0 ? hit[j] : 0];
        float f[kRowsPerLane][3];
        bool big = false;
#pragma unroll
        for (int j = 0; j < kRowsPerLane; ++j) {
            // a lane without a hit shades kFar (discarded below): on div180's
            // fast path like every hit
            const float normalised = div180(closest[j]);
            const float scalar = 255.0f - (normalised * 255.0f);
            f[j][0] = scalar * col[j].x;
            f[j][1] = scalar * col[j].y;
            f[j][2] = scalar * col[j].z;
            big |= !(fmaxf(fmaxf(f[j][0], f[j][1]), f[j][2]) < 2147483648.0f);
        }
        if (__ballot(big)) {
#pragma unroll
            for (int j = 0; j < kRowsPerLane; ++j) {
                const unsigned w = pack_bytes(cvt_i32_fast(f[j][0]), cvt_i32_fast(f[j][1]),
                                              cvt_i32_fast(f[j][2]));
                pix[j].x = hit[j] >= 0 ? (int)w : pix[j].x;
            }
        } else {
#pragma unroll
            for (int j = 0; j < kRowsPerLane; ++j) {
                int c[3];
#pragma unroll
                for (int k = 0; k < 3; ++k)
                    asm volatile("v_cvt_i32_f32 %0, %1" : "=v"(c[k]) : "v"(f[j][k]));
                const unsigned w = pack_bytes(c[0], c[1], c[2]);
                pix[j].x = hit[j] >= 0 ? (int)w : pix[j].x;
            }
        }
        return;
    }
#pragma unroll
    for (int j = 0; j < kRowsPerLane; ++j) pix[j] = int4v{0, 0, 0, 255};
    if (!any_hit) return;
    float4 col[kRowsPerLane];
#pragma unroll
    for (int j = 0; j < kRowsPerLane; ++j)  // kMode 4: no gather (diagnostics)
        col[j] = kMode == 4 ? make_float4(1.0f, 0.5f, 0.25f, 255.0f)
                            : colours[hit[j] >= 0 ? hit[j] : 0];
    // x86's (int) and v_cvt_i32_f32 agree except on NaN (INT32_MIN vs 0) and
    // f >= 2^31 (INT32_MIN vs INT32_MAX): one wave-uniform test picks the
    // raw converts, the per-channel fix-ups (cvt_i32_fast) run only when some
    // lane needs them.  Lanes without a hit shade kFar (discarded): on
    // div180's fast path like every hit.
    float f[kRowsPerLane][3];
    bool fix = false;
#pragma unroll
    for (int j = 0; j < kRowsPerLane; ++j) {
        const float normalised = div180(closest[j]);
        const float scalar = 255.0f - (normalised * 255.0f);
        f[j][0] = scalar * col[j].x;
        f[j][1] = scalar * col[j].y;
        f[j][2] = scalar * col[j].z;
        fix |= !(fmaxf(fmaxf(f[j][0], f[j][1]), f[j][2]) < 2147483648.0f) |
               __builtin_isunordered(f[j][0], f[j][1]) | __builtin_isunordered(f[j][2], f[j][2]);
    }
    if (__ballot(fix)) {
#pragma unroll
        for (int j = 0; j < kRowsPerLane; ++j) {
            const int4v c{cvt_i32_fast(f[j][0]), cvt_i32_fast(f[j][1]), cvt_i32_fast(f[j][2]), 255};
            pix[j] = hit[j] >= 0 ? c : pix[j];
        }
    } else {
#pragma unroll
        for (int j = 0; j < kRowsPerLane; ++j) {
            int c[3];
#pragma unroll
            for (int k = 0; k < 3; ++k)
                asm volatile("v_cvt_i32_f32 %0, %1" : "=v"(c[k]) : "v"(f[j][k]));
            pix[j] = hit[j] >= 0 ? int4v{c[0], c[1], c[2], 255} : pix[j];
        }
    }
}

// Store one lane's kRowsPerLane shaded pixels (rows kLaneRows apart) of the
// wave tile at (tile_x, tile_y), in the Texture format (MainState.cpp:
// 1026-1036, packed by shade_pixels) or int32x4.  `full`: the whole tile lies inside the frame band, so no
// per-lane bounds checks.
template <int kMode, int kFmt>
__device__ __forceinline__ void store_rows(const int4v* pix, int x, int y0, int width,
                                           int row_begin, int row_end, bool full,
                                           void* __restrict__ out) {
    const int64_t idx0 = (int64_t)(y0 - row_begin) * width + x;
    const int64_t row_step = (int64_t)kLaneRows * width;
#pragma unroll
    for (int j = 0; j < kRowsPerLane; ++j) {
        // kMode 3: everything but the stores (a store the compiler cannot drop)
        const bool store = kMode != 3 || pix[j].x == 0x7fffffff;
        if (full) {
            if (store) store_shaded<kFmt>(out, idx0 + j * row_step, pix[j]);
        } else {
            const int y = y0 + kLaneRows * j;
            if (x < width && y < row_end && store)
                store_shaded<kFmt>(out, idx0 + j * row_step, pix[j]);
        }
    }
}

// Tiles of one coarse bin: kCoarseW / kWaveTile x kCoarseH / kWaveTileH.
constexpr int kTilesX = kCoarseW / kWaveTile;
constexpr int kTilesY = kCoarseH / kWaveTileH;
constexpr int kTiles = kTilesX * kTilesY;
// tile words per candidate: kTileBits per tile, kTilesPerWord tiles a word
constexpr int kTmWords = (kTiles + kTilesPerWord - 1) / kTilesPerWord;
// ints per candidate slot of a coarse-bin list: the id, then the tile words
constexpr int kListStride = 1 + kTmWords;
static_assert(kTiles <= 16 && kTmWords <= 4, "tile words");

// Coarse binning with per-block classification: one wave per coarse bin.
// counts[cb] = -1 flags a frame whose scene data is not finite (prep's
// generation-stamped flag): the trace then runs the reference verbatim.
// (1) the ids whose box touches the coarse bin are compacted, in primitive
// order, into LDS (rounds of kRound); (2) the (candidate, tile) pairs are
// spread over the lanes, 16 lanes per candidate, each testing box overlap +
// classifier for every row block of its tile and OR-ing the bits (per
// block b: bit 2b keep, bit 2b+1 inside) into the candidate's LDS tile word;
// (3) candidates kept by some block are appended in order.  Output:
// counts[cb]; at lists + cb * kListStride * half_cap: half_cap ids, then
// tile word w of every candidate at [(1 + w) * half_cap ...].
#ifndef RT_C3_ABL
#define RT_C3_ABL 0  // diagnostics only: 1 = box scan + compaction, nothing classified or listed;
                     // 2 = as 1, every wave reading the same 64 boxes (L1-resident)
#endif
#ifndef RT_COARSE_CULL
#define RT_COARSE_CULL 10  // default of rt_debug_set_coarse_cull: bins with >= 10 sphere candidates
#endif
#ifndef RT_C3_ROUND
#define RT_C3_ROUND 64
#endif
#ifndef RT_C3_BATCH
#define RT_C3_BATCH 8
#endif
constexpr int kRound = RT_C3_ROUND;
static_assert(kTmWords == 1, "coarse depth cull: one tile word per candidate");
#ifndef RT_COARSE_WAVES
#define RT_COARSE_WAVES 6  // amdgpu_waves_per_eu floor for coarse3_kernel (0 = none): 80 VGPRs, 6 waves/SIMD (86 and 5 without; config 3 -0.4 us, config 5 dense -1.3%)
#endif
#if RT_COARSE_WAVES > 0
#define RT_COARSE_ATTR __attribute__((amdgpu_waves_per_eu(RT_COARSE_WAVES)))
#else
#define RT_COARSE_ATTR
#endif

// Coarse depth cull (`cull`): an upper bound on every pixel's final closest
// per wave tile, from the spheres that provably hit the WHOLE tile.  The
// trace computes, per pixel, dist2 = ((lx*lx + ly*ly) + kzw) - tca2 with
// lx = cx - x, ly = cy - y, then t0 = tca - sqrtf(r2 - dist2) (test_sph);
// every step is monotone under IEEE rounding, and |lx|, |ly| are largest at
// a tile edge, so the same operations on the tile's extreme |lx|, |ly| give
// dist2max >= dist2 and T = tca - sqrtf(r2 - dist2max) >= t0 at every pixel
// of the tile (exactly, no margin).  If dist2max <= r2 every pixel hits
// the sphere, and if t0 != 0 is guaranteed too (T < 0, or prep's lower
// bound tmin > 0) every pixel's closest ends <= T.  A sphere whose lower
// bound tmin is STRICTLY greater than the tile's smallest T then never wins
// a pixel of the tile (not even a tie: MainState.cpp:386-391 keeps the
// first of equal t), so its tile bits are cleared, and a candidate no tile
// keeps leaves the list.
// One-sided bounds of the correctly rounded sqrtf (x >= 0): v_sqrt_f32 is
// within 1 ulp of it on [2^-96, 2^126] (sqrt_rn_normal's +-1 ulp fix-up is
// exhaustively exact there, scripts/check_sqrt.hip), so +-2 ulp brackets it.
__device__ __forceinline__ float sqrt_lo_bound(float x) {  // <= sqrtf(x)
    if (!(x >= 0x1p-96f)) return 0.0f;
    if (!(x <= 0x1p126f)) return 0x1p63f;
    return __builtin_bit_cast(float, __builtin_bit_cast(int, __builtin_amdgcn_sqrtf(x)) - 2);
}
__device__ __forceinline__ float sqrt_hi_bound(float x) {  // >= sqrtf(x)
    if (!(x >= 0x1p-96f)) return 0x1p-48f;
    if (!(x <= 0x1p126f)) return INFINITY;
    return __builtin_bit_cast(float, __builtin_bit_cast(int, __builtin_amdgcn_sqrtf(x)) + 2);
}

// Upper bound (order key) of t0 over every pixel of the tile at (tx, ty),
// when the sphere provably hits all of them with t0 != 0; else ~0u.
__device__ __forceinline__ unsigned tile_cover_key(const SphRec& r, int tx, int ty) {
    const float xa = (float)tx, xb = (float)(tx + kWaveTile - 1);
    const float ya = (float)ty, yb = (float)(ty + kWaveTileH - 1);
    const float mx = fmaxf(fabsf(r.cx - xa), fabsf(r.cx - xb));
    const float my = fmaxf(fabsf(r.cy - ya), fabsf(r.cy - yb));
    const float a = (mx * mx) + (my * my);
    const float dist2 = (a + r.kzw) - r.tca2;
    if (!(dist2 <= r.r2)) return 0xffffffffu;  // some pixel may miss (or NaN)
    const float t = r.tca - sqrt_lo_bound(r.r2 - dist2);
    const bool nonzero = t < 0.0f || (t == t && r.tmin_key > order_key(0.0f));
    return nonzero ? order_key(t) : 0xffffffffu;
}

// Lower bound (order key) of t0 over the pixels of the tile at (tx, ty)
// that can hit the sphere: the same monotone operations on the tile's
// smallest |lx|, |ly| (0 when the centre's coordinate lies inside the
// tile's span) bound dist2 from below, so r2 - dist2 and thc from above.
// ~0u: no pixel of the tile hits (dist2 > r2 everywhere); 0: no bound.
__device__ __forceinline__ unsigned tile_low_key(const SphRec& r, int tx, int ty) {
    const float xa = (float)tx, xb = (float)(tx + kWaveTile - 1);
    const float ya = (float)ty, yb = (float)(ty + kWaveTileH - 1);
    const float lxa = r.cx - xa, lxb = r.cx - xb;  // lxa >= lxb
    const float lya = r.cy - ya, lyb = r.cy - yb;
    const float mx = (lxa >= 0.0f && lxb <= 0.0f) ? 0.0f : fminf(fabsf(lxa), fabsf(lxb));
    const float my = (lya >= 0.0f && lyb <= 0.0f) ? 0.0f : fminf(fabsf(lya), fabsf(lyb));
    const float a = (mx * mx) + (my * my);
    const float dist2 = (a + r.kzw) - r.tca2;
    if (dist2 > r.r2) return 0xffffffffu;
    const float t = r.tca - sqrt_hi_bound(r.r2 - dist2);
    return t == t ? order_key(t) : 0u;
}

__global__ void __launch_bounds__(64) RT_COARSE_ATTR coarse3_kernel(
    const int4* __restrict__ boxes, const Cls* __restrict__ cls,
    const SphRec* __restrict__ sph, int n_prims, int n_tri,
    int n_cx, const unsigned long long* __restrict__ row_masks,
    const unsigned long long* __restrict__ col_masks, int row_begin, int half_cap,
    const unsigned* __restrict__ nonfinite_flag, unsigned gen, int cull_min,
    int* __restrict__ counts, int* __restrict__ lists) {
    __shared__ int s_ids[kRound];
    __shared__ SphRec s_sph[kRound];
    __shared__ unsigned s_tkey[kTiles];  // per tile: smallest cover bound (order key)
    // read early (independent of the scan): a non-finite scene is handed to
    // the trace as count -1, so the trace's first scalar load tells it both
    const bool nonfinite = *nonfinite_flag == gen;
    __shared__ unsigned s_tm[kRound * kTmWords];
    __shared__ int4 s_box[kRound];
    __shared__ Cls s_cls[kRound];
    const int cb = blockIdx.x;
    const int lane = threadIdx.x;
    const int x0 = (cb % n_cx) * kCoarseW, x1 = x0 + kCoarseW - 1;
    const int y0 = row_begin + (cb / n_cx) * kCoarseH, y1 = y0 + kCoarseH - 1;
    int* out_id = lists + (int64_t)cb * kListStride * half_cap;
    int* out_tm = out_id + half_cap;
    int count = 0;   // appended to the output
    int staged = 0;  // ids in s_ids
    if (lane < kTiles) s_tkey[lane] = 0xffffffffu;
    // the depth cull runs in bins with at least cull_min sphere candidates (0: never)
    bool cull = false;
    constexpr int kBatch = RT_C3_BATCH;
    auto classify_round = [&](int n) {
        __builtin_amdgcn_wave_barrier();
        __atomic_signal_fence(__ATOMIC_SEQ_CST);
        // each candidate's box and classifier into LDS once
        for (int e = lane; e < n; e += 64) {
            const int id = s_ids[e];
#pragma unroll
            for (int w = 0; w < kTmWords; ++w) s_tm[e * kTmWords + w] = 0u;
            s_box[e] = boxes[id];
            s_cls[e] = cls[id];
            if (cull && id >= n_tri) s_sph[e] = sph[id - n_tri];
        }
        __builtin_amdgcn_wave_barrier();
        __atomic_signal_fence(__ATOMIC_SEQ_CST);
        for (int q0 = 0; q0 < n * kTiles; q0 += 64) {
            const int q = q0 + lane;
            if (q < n * kTiles) {
                const int c = q / kTiles, t = q % kTiles;
                const bool is_tri = s_ids[c] < n_tri;
                const int4 pb = s_box[c];
                const int tx = x0 + (t % kTilesX) * kWaveTile;
                const int ty = y0 + (t / kTilesX) * kWaveTileH;
                unsigned bits = 0u;
                bool keep = false, inside = false;
                if (pb.x <= tx + kWaveTile - 1 && pb.z >= tx && pb.y <= ty + kWaveTileH - 1 &&
                    pb.w >= ty)
                    classify(s_cls[c], is_tri, (float)tx, (float)ty, &keep, &inside);
                if (keep) bits = inside ? kTileMask : kKeepMask;
                if (cull && keep && !is_tri) {
                    const unsigned key = tile_cover_key(s_sph[c], tx, ty);
                    if (key != 0xffffffffu) atomicMin(&s_tkey[t], key);
                }
#if RT_ROWBITS == 1
                // a triangle's partial tile: classify each row block
                if (kBlocks > 1 && is_tri && keep && !inside) {
                    bits = 0u;
#pragma unroll
                    for (int b = 0; b < kBlocks; ++b) {
                        const int by = ty + b * kBlockH;
                        bool bk = false, bi = false;
                        if (pb.y <= by + kBlockH - 1 && pb.w >= by)
                            classify<kWaveTile, kBlockH>(s_cls[c], true, (float)tx, (float)by, &bk, &bi);
                        bits |= ((bk ? 1u : 0u) | (bk && bi ? 2u : 0u)) << (2 * b);
                    }
                }
#endif
                if (bits)
                    atomicOr(&s_tm[c * kTmWords + t / kTilesPerWord],
                             bits << (kTileBits * (t % kTilesPerWord)));
            }
        }
        __builtin_amdgcn_wave_barrier();
        __atomic_signal_fence(__ATOMIC_SEQ_CST);
        for (int e0 = 0; e0 < n; e0 += 64) {
            const int e = e0 + lane;
            unsigned tm[kTmWords];
            bool any = false;
#pragma unroll
            for (int w = 0; w < kTmWords; ++w) {
                tm[w] = e < n ? s_tm[e * kTmWords + w] : 0u;
                any |= tm[w] != 0u;
            }
            const unsigned long long m2 = __ballot(any);
            if (any) {
                const int pos = count + (int)__builtin_amdgcn_mbcnt_hi(
                    (unsigned)(m2 >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)m2, 0u));
                out_id[pos] = s_ids[e];
#pragma unroll
                for (int w = 0; w < kTmWords; ++w) out_tm[w * half_cap + pos] = (int)tm[w];
            }
            count += __popcll(m2);
        }
        __builtin_amdgcn_wave_barrier();
        __atomic_signal_fence(__ATOMIC_SEQ_CST);
    };
    // Stage the overlapping ids in primitive order (rounds of kRound).
    auto stage = [&](unsigned long long m, int chunk_base) {
        const int n_ov = __popcll(m);
        if (n_ov == 0) return;
        if (staged + n_ov > kRound) {
            if (RT_C3_ABL == 0) classify_round(staged);  // diag: 1 = scan only
            staged = 0;
        }
        if ((m >> lane) & 1ull) {
            const unsigned below = __builtin_amdgcn_mbcnt_hi(
                (unsigned)(m >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)m, 0u));
            s_ids[staged + (int)below] = chunk_base + lane;
        }
        staged += n_ov;
    };
    const int n_chunks = (n_prims + 63) / 64;
    if (row_masks) {
        // candidates = this bin row's chunk words AND this bin column's
        const unsigned long long* rw = row_masks + (int64_t)(cb / n_cx) * n_chunks;
        const unsigned long long* cw = col_masks + (int64_t)(cb % n_cx) * n_chunks;
        // lane l loads chunk c0 + l's two words; the nonzero chunks are
        // staged in order
        for (int c0 = 0; c0 < n_chunks; c0 += 64) {
            const int c = c0 + lane;
            const unsigned long long w = c < n_chunks ? rw[c] & cw[c] : 0ull;
            if (c0 == 0 && cull_min > 0) {
                // the gate: sphere candidates (ids >= n_tri) among the first
                // 4096 primitives, popcounts summed over the wave
                const int first = n_tri - 64 * c;
                const unsigned long long sph_bits =
                    first <= 0 ? ~0ull : first >= 64 ? 0ull : ~0ull << first;
                int n = __popcll(w & sph_bits);
#pragma unroll
                for (int off = 32; off > 0; off >>= 1) n += __shfl_xor(n, off);
                cull = n >= cull_min;
            }
            unsigned long long nz = __ballot(w != 0ull);
            while (nz) {
                const int l = __builtin_ctzll(nz);
                nz &= nz - 1ull;
                const unsigned long long m =
                    (unsigned long long)(unsigned)__builtin_amdgcn_readlane((int)(unsigned)w, l) |
                    ((unsigned long long)(unsigned)__builtin_amdgcn_readlane((int)(unsigned)(w >> 32), l) << 32);
                stage(m, (c0 + l) * 64);
            }
        }
    } else {
        cull = cull_min > 0;  // (count unknown before the scan)
        // scan every box (frames with too many bin rows + columns for masks)
        for (int base = 0; base < n_prims; base += 64 * kBatch) {
            int4 bb[kBatch];
#pragma unroll
            for (int k = 0; k < kBatch; ++k) {
                const int e = base + 64 * k + lane;
                bb[k] = e < n_prims ? boxes[RT_C3_ABL == 2 ? (e & 63) : e]
                                    : make_int4(1 << 30, 1 << 30, -(1 << 30), -(1 << 30));
            }
#pragma unroll
            for (int k = 0; k < kBatch; ++k) {
                const int4 q = bb[k];
                stage(__ballot(q.x <= x1 && q.z >= x0 && q.y <= y1 && q.w >= y0), base + 64 * k);
            }
        }
    }
    if (staged && RT_C3_ABL == 0) classify_round(staged);
    if (RT_C3_ABL != 0 && lane == 0) out_tm[0] = staged;  // keep the scan; lists stay empty
    // Depth cull (see tile_cover_key): once every candidate of the bin has
    // been classified, drop each sphere's tiles whose cover bound its tmin
    // strictly exceeds, and compact the list in place (in order: a kept
    // entry only moves down, past entries this wave has already read).
    if (cull && count > 0) {
        __builtin_amdgcn_wave_barrier();
        __atomic_signal_fence(__ATOMIC_SEQ_CST);
        const unsigned own = lane < kTiles ? s_tkey[lane] : 0xffffffffu;
        if (__ballot(own != 0xffffffffu)) {
            // the list this wave wrote is read back: its own stores are
            // ordered before the loads by a workgroup-scope fence (a wave
            // is its own workgroup here; agent scope would write back L2)
            __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
            int kept = 0;
            for (int e0 = 0; e0 < count; e0 += 64) {
                const int n = min(64, count - e0);
                const int e = e0 + lane;
                int id = -1;
                unsigned tm = 0u;
                if (e < count) {
                    id = out_id[e];
                    tm = (unsigned)out_tm[e];
                    if (id >= n_tri) s_sph[lane] = sph[id - n_tri];
                }
                s_ids[lane] = id;
                s_tm[lane] = tm;
                __builtin_amdgcn_wave_barrier();
                __atomic_signal_fence(__ATOMIC_SEQ_CST);
                // (candidate, tile) pairs over the lanes: a sphere leaves a
                // tile whose cover bound its tile-local t0 bound exceeds
                for (int q = lane; q < n * kTiles; q += 64) {
                    const int c = q / kTiles, t = q % kTiles;
                    const unsigned tkey = s_tkey[t];
                    if (s_ids[c] >= n_tri && tkey != 0xffffffffu &&
                        ((s_tm[c] >> (kTileBits * t)) & 1u)) {
                        const int tx = x0 + (t % kTilesX) * kWaveTile;
                        const int ty = y0 + (t / kTilesX) * kWaveTileH;
                        if (tile_low_key(s_sph[c], tx, ty) > tkey)
                            atomicAnd(&s_tm[c], ~(kTileMask << (kTileBits * t)));
                    }
                }
                __builtin_amdgcn_wave_barrier();
                __atomic_signal_fence(__ATOMIC_SEQ_CST);
                tm = s_tm[lane];
                __builtin_amdgcn_wave_barrier();
                __atomic_signal_fence(__ATOMIC_SEQ_CST);
                const bool any = e < count && tm != 0u;
                const unsigned long long m = __ballot(any);
                if (any) {
                    const int pos = kept + (int)__builtin_amdgcn_mbcnt_hi(
                        (unsigned)(m >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)m, 0u));
                    out_id[pos] = id;
                    out_tm[pos] = (int)tm;
                }
                kept += __popcll(m);
            }
            count = kept;
        }
    }
    if (lane == 0) counts[cb] = nonfinite ? -1 : count;
}

#if RT_TRACE_WAVES > 0
#define RT_TRACE_ATTR __attribute__((amdgpu_waves_per_eu(RT_TRACE_WAVES)))
#else
#define RT_TRACE_ATTR
#endif

#ifndef RT_XCD_REMAP
#define RT_XCD_REMAP 0  // trace: contiguous tile runs per XCD (T1 swizzle)
#endif
#ifndef RT_SPEC_BATCH
#define RT_SPEC_BATCH 0  // trace: first list batch loaded beside the count
#endif
#ifndef RT_DEPTH_CULL
#define RT_DEPTH_CULL 1  // skip spheres that cannot beat any lane's closest
#endif

// Wave-uniform order_key of the largest closest[] of the wave: per-lane max
// over its rows, then a DPP max to lane 63 (row_shr 1/2/4/8 within rows of
// 16, row_bcast 15/31 across them; shifted-in lanes read 0, the identity).
__device__ __forceinline__ unsigned wave_max_key(const float* closest) {
    float m = closest[0];
#pragma unroll
    for (int j = 1; j < kRowsPerLane; ++j) m = fmaxf(m, closest[j]);
    unsigned v = order_key(m);
    v = max(v, (unsigned)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xf, 0xf, false));
    v = max(v, (unsigned)__builtin_amdgcn_update_dpp(0, (int)v, 0x112, 0xf, 0xf, false));
    v = max(v, (unsigned)__builtin_amdgcn_update_dpp(0, (int)v, 0x114, 0xf, 0xf, false));
    v = max(v, (unsigned)__builtin_amdgcn_update_dpp(0, (int)v, 0x118, 0xf, 0xf, false));
    v = max(v, (unsigned)__builtin_amdgcn_update_dpp(0, (int)v, 0x142, 0xa, 0xf, false));
    v = max(v, (unsigned)__builtin_amdgcn_update_dpp(0, (int)v, 0x143, 0xc, 0xf, false));
    return (unsigned)__builtin_amdgcn_readlane((int)v, 63);
}

// One wave per kWaveTile x kWaveTileH tile, all candidate data on scalar
// loads: count, then ids and tile words 8 at a time, then the records of
// the candidates this tile keeps (in the reference's primitive order).
#ifndef RT_TRACE_WG
#define RT_TRACE_WG 1             // waves (tiles of one coarse bin) per trace workgroup
#endif
constexpr int kTraceWaves = RT_TRACE_WG;
#ifndef RT_TPW
#define RT_TPW 1                  // tiles of one coarse bin traced in turn by one wave
#endif
constexpr int kTilesPerWave = RT_TPW;
static_assert((kTilesX * kTilesY) % (kTraceWaves * kTilesPerWave) == 0,
              "trace workgroups must tile a coarse bin");
// Store hand-off (RT_LDS_STORE, with RT_TRACE_WG > 1): every wave of a
// trace workgroup leaves its shaded pixels in LDS and ends; the wave that
// finishes last issues the whole workgroup's frame stores, so only it waits
// for store acknowledgements at s_endpgm.  Measured slower on config 3
// (rejected variants); off.
#ifndef RT_LDS_STORE
#define RT_LDS_STORE 0
#endif
static_assert(!RT_LDS_STORE || kTilesPerWave == 1, "store hand-off: one tile per wave");

template <int kMode, int kFmt>
__global__ void __launch_bounds__(64 * kTraceWaves) RT_TRACE_ATTR trace3_kernel(
    SceneDev scene, const TriRec* __restrict__ tri, const SphRec* __restrict__ sph,
    const float4* __restrict__ colours, const int* __restrict__ counts,
    const int* __restrict__ lists, int half_cap, float4 dir, int width, int row_begin, int row_end, int n_tiles_x, int n_cx,
    int out_format, void* __restrict__ out) {
    // workgroup = kTraceWaves tiles of one coarse bin (independent waves on
    // one CU: the candidate records one wave loads are scalar-cache hits for
    // the others)
    constexpr int kGroups = (kTilesX * kTilesY) / (kTraceWaves * kTilesPerWave);
#if RT_XCD_REMAP
    // Workgroups are dealt round-robin over the 8 XCDs: give each XCD label
    // (b % 8) a contiguous run of tiles, so the 16 tiles of a coarse bin
    // share one L2 for its list and records (bijective for any grid size,
    // cdna_hip_programming.md T1).
    const int bid = [] {
        const int b = (int)blockIdx.x, nwg = (int)gridDim.x;
        const int q = nwg / 8, r = nwg % 8, xcd = b % 8;
        return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + b / 8;
    }();
#else
    const int bid = (int)blockIdx.x;
#endif
    const int cb = bid / kGroups;
    // wave-uniform by construction; readfirstlane tells the compiler, so the
    // per-candidate keep / inside bits stay in SGPRs (scalar branches)
    const int wave_id = (bid % kGroups) * kTraceWaves +
                        __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
#if RT_TIMELINE
    const int tile = blockIdx.x * kTraceWaves + (int)(threadIdx.x >> 6);
#endif
    const int lane = threadIdx.x & 63;
    const int n_tri = 12 * scene.n_cubes;
    (void)n_tiles_x;
    TL_MARK(tl0);
#if RT_TIMELINE
    const unsigned long long tlc0 = __builtin_amdgcn_s_memtime();
    unsigned tl1 = 0, tl2 = 0;
#endif
#if RT_LDS_STORE
    __shared__ int4v s_pix[kTraceWaves][kRowsPerLane][64];
    __shared__ int s_done;
    if (threadIdx.x == 0) s_done = 0;
    __syncthreads();
#endif
#pragma unroll 1
    for (int it = 0; it < kTilesPerWave; ++it) {
    const int t = wave_id * kTilesPerWave + it;
    const int rel_x = (cb % n_cx) * kCoarseW + (t % kTilesX) * kWaveTile;
    const int rel_y = (cb / n_cx) * kCoarseH + (t / kTilesX) * kWaveTileH;  // vs row_begin
    const int tile_x = rel_x, tile_y = row_begin + rel_y;
    const int x = tile_x + (lane % kWaveTile);
    const int y0 = tile_y + (lane / kWaveTile);
    // wave-uniform: tiles past the frame's right or bottom edge render nothing
    const bool tile_in = rel_x < width && rel_y < row_end - row_begin;
#if RT_LDS_STORE
    const int w_self = (int)(threadIdx.x >> 6);
#endif

    // the bin's count (-1: non-finite scene data, see coarse3_kernel) is the
    // wave's first data load
    const int count_raw = kMode == 1 ? 0 : counts[cb];
#if RT_SPEC_BATCH
    // the list's first batch of ids / tile words, loaded beside the count
    // (in bounds whatever the count: half_cap >= 8)
    const int* __restrict__ ids = lists + (int64_t)cb * kListStride * half_cap;
    const int* __restrict__ tms = ids + (1 + t / kTilesPerWord) * half_cap;  // this tile's word
    int idv[8], tmv[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        idv[k] = ids[k];
        tmv[k] = tms[k];
    }
#ifndef RT_SPEC_NOASM
    asm volatile("" ::"s"(count_raw), "s"(idv[0]), "s"(tmv[0]));
#endif
#endif
    if (tile_in && kMode == 0 && count_raw < 0) {
        // Non-finite scene data: run the reference algorithm verbatim.
#pragma unroll 1
        for (int j = 0; j < kRowsPerLane; ++j) {
            const int y = y0 + kLaneRows * j;
            int4v p = int4v{0, 0, 0, 255};
            if (x < width && y < row_end)
                p = collide_generic(scene, make_float4((float)x, (float)y, 0.0f, 1.0f), dir);
#if RT_LDS_STORE
            // store_rows stores shaded pixels: RGBA8 words packed in .x
            s_pix[w_self][j][lane] =
                kFmt == RT_FORMAT_RGBA8 ? int4v{(int)pack_rgba8(p), 0, 0, 0} : p;
#else
            if (x < width && y < row_end)
                store_fmt<kFmt>(out, (int64_t)(y - row_begin) * width + x, p);
#endif
        }
    } else {
    int4v pix[kRowsPerLane];  // assigned after the walk (not live during it)
    if (tile_in) {
    float closest[kRowsPerLane];
    int hit[kRowsPerLane];
    double py[kRowsPerLane];
    float pyf[kRowsPerLane];
#pragma unroll
    for (int j = 0; j < kRowsPerLane; ++j) {
        closest[j] = kFar;
        hit[j] = -1;
        py[j] = (double)(y0 + kLaneRows * j);
        pyf[j] = (float)(y0 + kLaneRows * j);
    }
    const double px = (double)x;
    const float pxf = (float)x;
#if RT_DEPTH_CULL
    // order_key of the largest `closest` in the tile, refreshed lazily
    unsigned tile_max_key = order_key(kFar);
    bool dirty = false;
#endif
    const int count = count_raw < 0 ? 0 : count_raw;
#if !RT_SPEC_BATCH
    const int* __restrict__ ids = lists + (int64_t)cb * kListStride * half_cap;
    const int* __restrict__ tms = ids + (1 + t / kTilesPerWord) * half_cap;  // this tile's word
#endif
    const int tm_shift = kTileBits * (t % kTilesPerWord);
#if RT_TIMELINE
    tl1 = rt_now();
#endif
    for (int i0 = 0; i0 < count; i0 += 8) {
#if RT_SPEC_BATCH
        if (i0 > 0) {
#else
        int idv[8], tmv[8];
        {
#endif
#pragma unroll
            for (int k = 0; k < 8; ++k) {
                idv[k] = ids[i0 + k];  // half_cap is a multiple of 8 past the count
                tmv[k] = tms[i0 + k];
            }
        }
        const int n = min(8, count - i0);
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            if (k >= n) break;
            const unsigned bits = ((unsigned)tmv[k] >> tm_shift) & kTileMask;
            if (!(bits & kKeepMask)) continue;
            const int p = idv[k];
            if (kMode == 2) {
                hit[0] = hit[0] > p ? hit[0] : -1;
                continue;
            }
            if (p < n_tri) {
                const TriRec r = tri[p];
                asm volatile("" ::"s"(r.p0), "s"(r.p1), "s"(r.dz));
                test_tri<row_skip<kFmt>()>(r, p / 12, bits, px, py, closest, hit);
            } else {
                const SphRec r = sph[p - n_tri];
#if RT_DEPTH_CULL
                // t0 >= tmin >= every closest: no lane can take it (strict <)
                if (dirty) {
                    tile_max_key = wave_max_key(closest);
                    dirty = false;
                }
                if (r.tmin_key >= tile_max_key) continue;
#endif
                test_sph<row_skip<kFmt>()>(r, scene.n_cubes + (p - n_tri), bits, pxf, pyf, closest,
                                           hit);
            }
#if RT_DEPTH_CULL
            dirty = true;
#endif
        }
    }
#if RT_TIMELINE
    tl2 = rt_now();
#endif
    shade_pixels<kMode, kFmt>(colours, closest, hit, pix);
    } else {  // outside the frame: nothing is stored
#pragma unroll
        for (int j = 0; j < kRowsPerLane; ++j)
            pix[j] = int4v{kFmt == RT_FORMAT_RGBA8 ? (int)0xFF000000u : 0, 0, 0, 255};
    }
#if RT_LDS_STORE
#pragma unroll
    for (int j = 0; j < kRowsPerLane; ++j) s_pix[w_self][j][lane] = pix[j];
#else
    if (tile_in) {
        const bool full = rel_x + kWaveTile <= width && tile_y + kWaveTileH <= row_end;
        store_rows<kMode, kFmt>(pix, x, y0, width, row_begin, row_end, full, out);
    }
#endif
    }  // finite scene
#if RT_LDS_STORE
    // then the last wave of the workgroup stores every tile
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");  // every lane's deposit
    int prev = 0;
    if (lane == 0)
        prev = __hip_atomic_fetch_add(&s_done, 1, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_WORKGROUP);
    prev = __builtin_amdgcn_readfirstlane(prev);
    if (prev == kTraceWaves - 1) {  // the other waves' deposits are complete
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
#pragma unroll 1
        for (int w = 0; w < kTraceWaves; ++w) {
            const int tw = (bid % kGroups) * kTraceWaves + w;
            const int wx = (cb % n_cx) * kCoarseW + (tw % kTilesX) * kWaveTile;
            const int wy = (cb / n_cx) * kCoarseH + (tw / kTilesX) * kWaveTileH;
            if (wx >= width || wy >= row_end - row_begin) continue;  // uniform
            int4v q[kRowsPerLane];
#pragma unroll
            for (int j = 0; j < kRowsPerLane; ++j) q[j] = s_pix[w][j][lane];
            const bool full = wx + kWaveTile <= width && row_begin + wy + kWaveTileH <= row_end;
            store_rows<kMode, kFmt>(q, wx + (lane % kWaveTile), row_begin + wy + (lane / kWaveTile),
                                    width, row_begin, row_end, full, out);
        }
    }
#endif
    }  // tiles of this wave
#if RT_TIMELINE
    {
        const unsigned tl3 = rt_now();
        const unsigned long long tlc3 = __builtin_amdgcn_s_memtime();
        if (lane == 0) {
            unsigned* o = g_timeline + 8 * (int64_t)tile;
            o[0] = tl0; o[1] = tl1; o[2] = tl2; o[3] = tl3;
            o[4] = (unsigned)tlc0; o[5] = (unsigned)tlc3;
            o[6] = __builtin_amdgcn_s_getreg((31 << 11) | 4);
            o[7] = __builtin_amdgcn_s_getreg((31 << 11) | 20);
        }
    }
#endif
}

// Small scenes (at most 64 x RT_SMALL_CHUNKS primitives, that many prep
// chunks): no coarse kernel and no candidate lists.  Each tile wave ANDs its
// bin row's and bin column's mask words per chunk (the candidates, in
// primitive order), lets lane i classify candidate 64 c + i against the tile
// exactly as coarse3_kernel does, and walks the kept candidates from the
// ballots, chunk by chunk.  Saves the coarse launch and
// one kernel boundary, which dominate small frames (config 2).
#ifndef RT_SMALL_CHUNKS
#define RT_SMALL_CHUNKS 8  // the small-scene path takes scenes of up to 64 x this many primitives
#endif
template <int kFmt, int kChunks>
__global__ void __launch_bounds__(64) RT_TRACE_ATTR trace_small_kernel(
    const unsigned long long* __restrict__ row_masks,
    const unsigned long long* __restrict__ col_masks, const int4* __restrict__ boxes,
    const Cls* __restrict__ cls, const TriRec* __restrict__ tri, const SphRec* __restrict__ sph,
    const float4* __restrict__ colours, const unsigned* __restrict__ nonfinite_flag,
    unsigned gen, int n_cubes, int n_cx, int n_chunks, int width, int row_begin, int row_end,
    SceneDev scene, float4 dir, void* __restrict__ out) {
    const int bid = (int)blockIdx.x;
    const int cb = bid / kTiles;
    const int t = __builtin_amdgcn_readfirstlane(bid % kTiles);
    const int lane = threadIdx.x & 63;
    const int n_tri = 12 * n_cubes;
    const int rel_x = (cb % n_cx) * kCoarseW + (t % kTilesX) * kWaveTile;
    const int rel_y = (cb / n_cx) * kCoarseH + (t / kTilesX) * kWaveTileH;
    if (!(rel_x < width && rel_y < row_end - row_begin)) return;  // outside: no stores
    const int tile_x = rel_x, tile_y = row_begin + rel_y;
    const int x = tile_x + (lane % kWaveTile);
    const int y0 = tile_y + (lane / kWaveTile);
    unsigned long long cand[kChunks];
#pragma unroll
    for (int c = 0; c < kChunks; ++c)
        cand[c] = c < n_chunks ? row_masks[(int64_t)(cb / n_cx) * n_chunks + c] &
                                     col_masks[(int64_t)(cb % n_cx) * n_chunks + c]
                               : 0ull;
    const bool nonfinite = *nonfinite_flag == gen;
    int4v pix[kRowsPerLane];
    if (nonfinite) {  // the reference algorithm verbatim (see trace3_kernel)
#pragma unroll 1
        for (int j = 0; j < kRowsPerLane; ++j) {
            const int y = y0 + kLaneRows * j;
            if (x < width && y < row_end)
                store_fmt<kFmt>(out, (int64_t)(y - row_begin) * width + x,
                                collide_generic(scene, make_float4((float)x, (float)y, 0.0f, 1.0f),
                                                dir));
        }
        return;
    }
    // lane i: candidate 64 c + i against this tile (coarse3_kernel's test)
    unsigned long long keep[kChunks], inside[kChunks];
#pragma unroll
    for (int c = 0; c < kChunks; ++c) {
        const int q = 64 * c + lane;
        bool keep_l = false, inside_l = false;
        if ((cand[c] >> lane) & 1ull) {
            const int4 pb = boxes[q];
            const int tx = tile_x, ty = tile_y;
            if (pb.x <= tx + kWaveTile - 1 && pb.z >= tx && pb.y <= ty + kWaveTileH - 1 &&
                pb.w >= ty)
                classify(cls[q], q < n_tri, (float)tx, (float)ty, &keep_l, &inside_l);
        }
        keep[c] = __ballot(keep_l);
        inside[c] = __ballot(keep_l && inside_l);
    }
    float closest[kRowsPerLane];
    int hit[kRowsPerLane];
    double py[kRowsPerLane];
    float pyf[kRowsPerLane];
#pragma unroll
    for (int j = 0; j < kRowsPerLane; ++j) {
        closest[j] = kFar;
        hit[j] = -1;
        py[j] = (double)(y0 + kLaneRows * j);
        pyf[j] = (float)(y0 + kLaneRows * j);
    }
    const double px = (double)x;
    const float pxf = (float)x;
#if RT_DEPTH_CULL
    unsigned tile_max_key = order_key(kFar);
    bool dirty = false;
#endif
#pragma unroll
    for (int c = 0; c < kChunks; ++c)
    while (keep[c]) {  // kept candidates in primitive order
        const int b = __builtin_ctzll(keep[c]);
        keep[c] &= keep[c] - 1ull;
        const int p = 64 * c + b;
        const unsigned bits = ((inside[c] >> b) & 1ull) ? kTileMask : kKeepMask;
        if (p < n_tri) {
            const TriRec r = tri[p];
            asm volatile("" ::"s"(r.p0), "s"(r.p1), "s"(r.dz));
            test_tri<row_skip<kFmt>()>(r, p / 12, bits, px, py, closest, hit);
        } else {
            const SphRec r = sph[p - n_tri];
#if RT_DEPTH_CULL
            if (dirty) {
                tile_max_key = wave_max_key(closest);
                dirty = false;
            }
            if (r.tmin_key >= tile_max_key) continue;
#endif
            test_sph<row_skip<kFmt>()>(r, n_cubes + (p - n_tri), bits, pxf, pyf, closest, hit);
        }
#if RT_DEPTH_CULL
        dirty = true;
#endif
    }
    shade_pixels<0, kFmt>(colours, closest, hit, pix);
    const bool full = rel_x + kWaveTile <= width && tile_y + kWaveTileH <= row_end;
    store_rows<0, kFmt>(pix, x, y0, width, row_begin, row_end, full, out);
}

// fp32 self-test: the device's sqrtf and '/' must be correctly rounded.
__global__ void fp32_selftest_kernel(const float* in, int n, float* out_sqrt, float* out_div) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    out_sqrt[i] = sqrtf(in[i]);
    out_div[i] = in[i] / 180.0f;
}

}  // namespace

// ===========================================================================
// Host side
// ===========================================================================
struct rt_ctx {
    int device = 0;
    hipStream_t stream = nullptr;
    // workspace (grow-only)
    void* scene_buf = nullptr;  size_t scene_cap = 0;   // host-API scene copy
    void* origin_buf = nullptr; size_t origin_cap = 0;  // host-API explicit origins
    void* out_buf = nullptr;    size_t out_cap = 0;     // host-API frame
    void* rec_buf = nullptr;    size_t rec_cap = 0;     // TriRec/SphRec/boxes/flag
    void* list_buf = nullptr;   size_t list_cap = 0;    // coarse-bin candidate lists
    unsigned* flag = nullptr;   // non-finite scene flag (generation-stamped)
    unsigned gen = 0;
    int trace_mode = 0;  // diagnostics ablation, see trace3_kernel
    // coarse lists take 4 B x kListStride x (primitives + 16) per 64x64 bin; a frame whose
    // lists would exceed this is rendered as internal row bands
    int64_t list_budget = (int64_t)4 << 30;
    bool bin_masks = RT_BIN_MASKS != 0;  // separable bin masks (false: coarse scans every box)
    bool small_path = true;  // <= 64 x RT_SMALL_CHUNKS primitives: trace_small_kernel
    // coarse depth cull of sphere candidates in bins with at least this many
    // candidates (0 = off)
    int coarse_cull = RT_COARSE_CULL;
    hipEvent_t ev[4] = {nullptr, nullptr, nullptr, nullptr};
    // profiling: per render, start/stop events of the prep, coarse and trace
    // kernels, attached to the kernels' own dispatch packets
    bool profile = false;
    std::vector<hipEvent_t> prof_events;  // a pool: created once, reused
    std::vector<unsigned char> prof_skipped;  // per event pair: no kernel ran (0 ms)
    size_t prof_used = 0;                 // events holding this batch's timestamps
    int32_t prof_count = 0;
};

namespace rt_internal {
int ctx_device(const rt_ctx* ctx) { return ctx->device; }
hipStream_t ctx_stream(const rt_ctx* ctx) { return ctx->stream; }
}  // namespace rt_internal

namespace {

size_t align_up(size_t v, size_t a) { return (v + a - 1) / a * a; }

int ensure(void** buf, size_t* cap, size_t need) {
    if (need <= *cap) return RT_OK;
    if (*buf) {
        (void)hipFree(*buf);
        *buf = nullptr;
        *cap = 0;
    }
    size_t n = align_up(need + need / 4, 1 << 16);
    if (hipMalloc(buf, n) != hipSuccess) {
        *buf = nullptr;
        return RT_ERR_OUT_OF_MEMORY;
    }
    *cap = n;
    return RT_OK;
}

bool binned_ok(const float d[4], const float* origins) {
    return origins == nullptr && d[0] == 0.0f && d[1] == 0.0f && d[2] != 0.0f &&
           std::isfinite(d[2]) && std::isfinite(d[3]);
}

int check_args(const rt_scene* s, int32_t width, int32_t height, int32_t row_begin,
               int32_t row_end, int32_t fmt) {
    if (!s || width <= 0 || height <= 0 || row_begin < 0 || row_end > height ||
        row_begin >= row_end)
        return RT_ERR_INVALID_ARG;
    if (width > (1 << 24) || height > (1 << 24)) return RT_ERR_INVALID_ARG;  // exact float coords
    if (s->num_spheres < 0 || s->num_cubes < 0 || s->num_lights < 0) return RT_ERR_INVALID_ARG;
    if (s->num_spheres > 0 && (!s->sphere_origins || !s->sphere_radius || !s->sphere_colours))
        return RT_ERR_INVALID_ARG;
    if (s->num_cubes > 0 && (!s->cube_vertices || !s->cube_colours)) return RT_ERR_INVALID_ARG;
    if ((int64_t)12 * s->num_cubes + s->num_spheres > (int64_t)1 << 30) return RT_ERR_INVALID_ARG;
    if (fmt != RT_FORMAT_I32X4 && fmt != RT_FORMAT_RGBA8) return RT_ERR_INVALID_ARG;
    return RT_OK;
}

#define HIP_TRY(x)                                    \
    do {                                              \
        if ((x) != hipSuccess) return RT_ERR_HIP;     \
    } while (0)

// Launch `kernel` on `stream`; with profiling events, through
// hipExtLaunchKernelGGL so the start/stop timestamps are the kernel's own
// (no extra queue packets between the kernels).
template <typename K, typename... A>
int launch_k(K kernel, dim3 grid, dim3 block, hipStream_t stream, const hipEvent_t* ev,
             A... args) {
    if (ev)
        hipExtLaunchKernelGGL(kernel, grid, block, 0, stream, ev[0], ev[1], 0, args...);
    else
        kernel<<<grid, block, 0, stream>>>(args...);
    return hipGetLastError() == hipSuccess ? RT_OK : RT_ERR_HIP;
}

// A profiled kernel slot that runs nothing: flagged, so it reads 0 ms.
// (Recording the two events back to back would time the marker packets
// themselves, ~5 us, not a kernel.)
int skip_k(rt_ctx* ctx, const hipEvent_t* ev) {
    if (!ev) return RT_OK;
    ctx->prof_skipped[(size_t)(ev - ctx->prof_events.data()) / 2] = 1;
    return RT_OK;
}

// Enqueue one render of rows [row_begin, row_end) on `stream`.  All scene
// pointers are device pointers.
int launch(rt_ctx* ctx, const rt_scene* s, const float d[4], const float* origins,
           int32_t width, int32_t row_begin, int32_t row_end, int32_t fmt,
           int32_t path, void* out, hipStream_t stream, int32_t* used_path) {
    SceneDev sd{reinterpret_cast<const float4*>(s->sphere_origins), s->sphere_radius,
                reinterpret_cast<const float4*>(s->sphere_colours),
                reinterpret_cast<const float4*>(s->cube_vertices),
                reinterpret_cast<const float4*>(s->cube_colours), s->num_spheres, s->num_cubes};
    const float4 dir = make_float4(d[0], d[1], d[2], d[3]);
    const int32_t rows = row_end - row_begin;
    const bool can_bin = binned_ok(d, origins);
    if (path == RT_PATH_BINNED && !can_bin) return RT_ERR_UNSUPPORTED;
    const bool use_bin = path == RT_PATH_BINNED || (path == RT_PATH_AUTO && can_bin);
    if (used_path) *used_path = use_bin ? RT_PATH_BINNED : RT_PATH_GENERIC;
    if (use_bin) {
        // Bound the candidate-list workspace: split into bands of whole
        // coarse rows, each a band render (bin masks per band),
        // in order on the same stream.
        const int64_t n_prims = 12 * (int64_t)s->num_cubes + s->num_spheres;
        const int64_t row_bytes =
            4 * kListStride * ((n_prims + 7) / 8 * 8 + 8) * ((width + kCoarseW - 1) / kCoarseW);
        const int64_t n_cy = (rows + kCoarseH - 1) / kCoarseH;
        if (n_cy > 1 && row_bytes * n_cy > ctx->list_budget) {
            const int64_t per = std::max<int64_t>(1, ctx->list_budget / row_bytes) * kCoarseH;
            const size_t px_bytes = fmt == RT_FORMAT_I32X4 ? 16 : 4;
            const int32_t prof_count0 = ctx->prof_count;
            for (int64_t rb = row_begin; rb < row_end; rb += per) {
                const int32_t re = (int32_t)std::min<int64_t>(rb + per, row_end);
                char* dst = static_cast<char*>(out) + (size_t)(rb - row_begin) * width * px_bytes;
                const int rc = launch(ctx, s, d, origins, width, (int32_t)rb, re, fmt, path, dst,
                                      stream, nullptr);
                if (rc) return rc;
            }
            if (ctx->profile) ctx->prof_count = prof_count0 + 1;  // one render, summed bands
            return RT_OK;
        }
    }
    const hipEvent_t* pe = nullptr;  // 6 events: prep, coarse, trace (start, stop)
    if (ctx->profile) {
        while (ctx->prof_events.size() < ctx->prof_used + 6) {
            hipEvent_t e;
            HIP_TRY(hipEventCreate(&e));
            ctx->prof_events.push_back(e);
        }
        ctx->prof_skipped.resize(ctx->prof_events.size() / 2);
        for (int k = 0; k < 3; ++k) ctx->prof_skipped[ctx->prof_used / 2 + k] = 0;
        pe = &ctx->prof_events[ctx->prof_used];
        ctx->prof_used += 6;
        ++ctx->prof_count;
    }
    const hipEvent_t* pe_prep = pe ? pe : nullptr;
    const hipEvent_t* pe_coarse = pe ? pe + 2 : nullptr;
    const hipEvent_t* pe_trace = pe ? pe + 4 : nullptr;
    int rc;
    if (!use_bin) {
        const int64_t n = (int64_t)width * rows;
        const int64_t blocks = std::min<int64_t>((n + kThreads - 1) / kThreads, (int64_t)1 << 20);
        if ((rc = skip_k(ctx, pe_prep)) || (rc = skip_k(ctx, pe_coarse))) return rc;
        return launch_k(generic_kernel, dim3((unsigned)blocks), dim3(kThreads), stream, pe_trace,
                        sd, dir, reinterpret_cast<const float4*>(origins), width, row_begin,
                        row_end, fmt, out);
    }
    const int n_tri = 12 * s->num_cubes;
    const int n_prims = n_tri + s->num_spheres;
    const int n_cx = (width + kCoarseW - 1) / kCoarseW;
    const int n_cy = (rows + kCoarseH - 1) / kCoarseH;
    const int64_t n_coarse64 = (int64_t)n_cx * n_cy;
    const int n_tiles_x = (width + kWaveTile - 1) / kWaveTile;
    const int64_t n_wgs = n_coarse64 * (kTilesX * kTilesY / (kTraceWaves * kTilesPerWave));
    // one trace work-item per 64 x kTraceWaves; AQL grid sizes are 32-bit
    if (n_wgs * 64 * kTraceWaves > (int64_t)UINT32_MAX) return RT_ERR_INVALID_ARG;
    const int n_coarse = (int)n_coarse64;
    // per coarse bin: candidate ids, then each tile word (half_cap each,
    // padded by 8 so the trace's 8-wide scalar reads stay inside the bin)
    const int half_cap = (n_prims + 7) / 8 * 8 + 8;

    const size_t tri_off = 0;
    const size_t sph_off = align_up(sizeof(TriRec) * (size_t)n_tri, 256);
    const size_t box_off = sph_off + align_up(sizeof(SphRec) * (size_t)s->num_spheres, 256);
    const size_t cls_off = box_off + align_up(sizeof(int4) * (size_t)n_prims, 256);
    const size_t col_off = cls_off + align_up(sizeof(Cls) * (size_t)n_prims, 256);
    const size_t cnt_off =
        col_off + align_up(sizeof(float4) * (size_t)(s->num_cubes + s->num_spheres), 256);
    const int n_chunks = (n_prims + kPrepThreads - 1) / kPrepThreads;
    const bool use_masks = ctx->bin_masks && (int64_t)n_cx + n_cy <= kMaskBinsMax;
    const size_t mask_off = cnt_off + align_up(sizeof(int) * (size_t)n_coarse, 256);
    const size_t n_mask_words = use_masks ? (size_t)n_chunks * (size_t)(n_cx + n_cy) : 0;
    const size_t rec_need = mask_off + align_up(sizeof(unsigned long long) * n_mask_words, 256);
    rc = ensure(&ctx->rec_buf, &ctx->rec_cap, rec_need);
    if (rc) return rc;
    const size_t list_need = sizeof(int) * kListStride * (size_t)half_cap * (size_t)n_coarse + 256;
    rc = ensure(&ctx->list_buf, &ctx->list_cap, list_need);
    if (rc) return rc;
    char* base = static_cast<char*>(ctx->rec_buf);
    TriRec* tri = reinterpret_cast<TriRec*>(base + tri_off);
    SphRec* sph = reinterpret_cast<SphRec*>(base + sph_off);
    int4* boxes = reinterpret_cast<int4*>(base + box_off);
    Cls* clsv = reinterpret_cast<Cls*>(base + cls_off);
    float4* colours = reinterpret_cast<float4*>(base + col_off);
    int* counts = reinterpret_cast<int*>(base + cnt_off);
    unsigned long long* row_masks =
        use_masks ? reinterpret_cast<unsigned long long*>(base + mask_off) : nullptr;
    unsigned long long* col_masks = use_masks ? row_masks + (size_t)n_chunks * n_cy : nullptr;
    int* lists = static_cast<int*>(ctx->list_buf);
    // generation-stamped non-finite flag: no per-launch memset needed
    if (++ctx->gen == 0) {
        HIP_TRY(hipMemsetAsync(ctx->flag, 0, sizeof(unsigned), stream));
        ctx->gen = 1;
    }

    if (n_prims > 0 && n_chunks <= RT_SMALL_CHUNKS && use_masks && ctx->small_path &&
        ctx->trace_mode == 0) {
        rc = launch_k(prep_kernel, dim3((unsigned)n_chunks), dim3(kPrepThreads), stream, pe_prep, sd, dir, width,
                      row_begin, row_end, tri, sph, boxes, clsv, colours, ctx->flag, ctx->gen,
                      row_masks, col_masks, n_cx, n_cy);
        if (rc) return rc;
        if ((rc = skip_k(ctx, pe_coarse))) return rc;
        // the instance with the fewest chunk slots that holds n_chunks
        const bool i32 = fmt == RT_FORMAT_I32X4;
        auto small = n_chunks == 1   ? (i32 ? trace_small_kernel<RT_FORMAT_I32X4, 1>
                                            : trace_small_kernel<RT_FORMAT_RGBA8, 1>)
                     : n_chunks == 2 ? (i32 ? trace_small_kernel<RT_FORMAT_I32X4, 2>
                                            : trace_small_kernel<RT_FORMAT_RGBA8, 2>)
                     : n_chunks <= 4 || RT_SMALL_CHUNKS <= 4
                         ? (i32 ? trace_small_kernel<RT_FORMAT_I32X4, 4>
                                : trace_small_kernel<RT_FORMAT_RGBA8, 4>)
                         : (i32 ? trace_small_kernel<RT_FORMAT_I32X4, RT_SMALL_CHUNKS>
                                : trace_small_kernel<RT_FORMAT_RGBA8, RT_SMALL_CHUNKS>);
        return launch_k(small, dim3((unsigned)(n_coarse64 * kTiles)), dim3(64), stream, pe_trace,
                        (const unsigned long long*)row_masks, (const unsigned long long*)col_masks,
                        (const int4*)boxes, (const Cls*)clsv, (const TriRec*)tri,
                        (const SphRec*)sph, (const float4*)colours, (const unsigned*)ctx->flag,
                        ctx->gen, s->num_cubes, n_cx, n_chunks, width, row_begin, row_end, sd,
                        dir, out);
    }
    if (n_prims > 0) {
        rc = launch_k(prep_kernel, dim3((unsigned)n_chunks), dim3(kPrepThreads), stream, pe_prep,
                      sd, dir, width, row_begin, row_end, tri, sph, boxes, clsv, colours,
                      ctx->flag, ctx->gen, row_masks, col_masks, n_cx, n_cy);
        if (rc) return rc;
        rc = launch_k(coarse3_kernel, dim3((unsigned)n_coarse), dim3(64), stream, pe_coarse,
                      (const int4*)boxes, (const Cls*)clsv, (const SphRec*)sph, n_prims, n_tri,
                      n_cx, (const unsigned long long*)row_masks,
                      (const unsigned long long*)col_masks, row_begin, half_cap,
                      (const unsigned*)ctx->flag, ctx->gen, ctx->coarse_cull, counts, lists);
        if (rc) return rc;
    } else {
        if ((rc = skip_k(ctx, pe_prep))) return rc;
        HIP_TRY(hipMemsetAsync(counts, 0, sizeof(int) * (size_t)n_coarse, stream));
        if ((rc = skip_k(ctx, pe_coarse))) return rc;
    }
    auto kern = fmt == RT_FORMAT_I32X4
                    ? (ctx->trace_mode == 1   ? trace3_kernel<1, RT_FORMAT_I32X4>
                       : ctx->trace_mode == 2 ? trace3_kernel<2, RT_FORMAT_I32X4>
                       : ctx->trace_mode == 3 ? trace3_kernel<3, RT_FORMAT_I32X4>
                       : ctx->trace_mode == 4 ? trace3_kernel<4, RT_FORMAT_I32X4>
                                              : trace3_kernel<0, RT_FORMAT_I32X4>)
                    : (ctx->trace_mode == 1   ? trace3_kernel<1, RT_FORMAT_RGBA8>
                       : ctx->trace_mode == 2 ? trace3_kernel<2, RT_FORMAT_RGBA8>
                       : ctx->trace_mode == 3 ? trace3_kernel<3, RT_FORMAT_RGBA8>
                       : ctx->trace_mode == 4 ? trace3_kernel<4, RT_FORMAT_RGBA8>
                                              : trace3_kernel<0, RT_FORMAT_RGBA8>);
    return launch_k(kern, dim3((unsigned)n_wgs), dim3(64 * kTraceWaves), stream, pe_trace, sd,
                    (const TriRec*)tri, (const SphRec*)sph, (const float4*)colours,
                    (const int*)counts, (const int*)lists, half_cap, dir, width, row_begin, row_end, n_tiles_x, n_cx, fmt, out);
}

}  // namespace

extern "C" {

const char* rt_error_string(int status) {
    switch (status) {
    case RT_OK: return "success";
    case RT_ERR_INVALID_ARG: return "invalid argument";
    case RT_ERR_NO_DEVICE: return "no HIP device available";
    case RT_ERR_HIP: return "HIP runtime error";
    case RT_ERR_OUT_OF_MEMORY: return "device out of memory";
    case RT_ERR_UNSUPPORTED: return "requested path unsupported for these rays";
    default: return "unknown error";
    }
}

int rt_init(int device_ordinal, rt_ctx** out_ctx) {
    if (!out_ctx) return RT_ERR_INVALID_ARG;
    *out_ctx = nullptr;
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) return RT_ERR_NO_DEVICE;
    if (device_ordinal < 0 || device_ordinal >= n) return RT_ERR_INVALID_ARG;
    if (hipSetDevice(device_ordinal) != hipSuccess) return RT_ERR_HIP;
    rt_ctx* ctx = new rt_ctx();
    ctx->device = device_ordinal;
    if (hipStreamCreateWithFlags(&ctx->stream, hipStreamNonBlocking) != hipSuccess) {
        delete ctx;
        return RT_ERR_HIP;
    }
    for (auto& e : ctx->ev) {
        if (hipEventCreate(&e) != hipSuccess) {
            rt_destroy(ctx);
            return RT_ERR_HIP;
        }
    }
    // [0] non-finite flag
    if (hipMalloc(&ctx->flag, 4 * sizeof(unsigned)) != hipSuccess ||
        hipMemset(ctx->flag, 0, 4 * sizeof(unsigned)) != hipSuccess) {
        rt_destroy(ctx);
        return RT_ERR_OUT_OF_MEMORY;
    }
    *out_ctx = ctx;
    return RT_OK;
}

void rt_destroy(rt_ctx* ctx) {
    if (!ctx) return;
    (void)hipSetDevice(ctx->device);
    if (ctx->stream) (void)hipStreamSynchronize(ctx->stream);
    for (void* p : {ctx->scene_buf, ctx->origin_buf, ctx->out_buf, ctx->rec_buf, ctx->list_buf,
                    static_cast<void*>(ctx->flag)})
        if (p) (void)hipFree(p);
    for (auto& e : ctx->ev)
        if (e) (void)hipEventDestroy(e);
    for (auto e : ctx->prof_events) (void)hipEventDestroy(e);
    if (ctx->stream) (void)hipStreamDestroy(ctx->stream);
    delete ctx;
}

int rt_render_path(rt_ctx* ctx, const rt_scene* scene, const float ray_dir[4],
                   const float* ray_origins, int32_t width, int32_t height, int32_t row_begin,
                   int32_t row_end, int32_t out_format, int32_t path, void* host_out,
                   rt_timing* timing) {
    const auto t0 = std::chrono::steady_clock::now();
    if (!ctx || !ray_dir || !host_out) return RT_ERR_INVALID_ARG;
    int rc = check_args(scene, width, height, row_begin, row_end, out_format);
    if (rc) return rc;
    if (path < RT_PATH_AUTO || path > RT_PATH_GENERIC) return RT_ERR_INVALID_ARG;
    HIP_TRY(hipSetDevice(ctx->device));
    const int32_t rows = row_end - row_begin;
    const size_t ns = (size_t)scene->num_spheres, nc = (size_t)scene->num_cubes;
    // one device copy of the flattened scene (MainState.cpp:666-743, 759-838)
    const size_t o_so = 0, o_sr = align_up(16 * ns, 256), o_sc = o_sr + align_up(4 * ns, 256),
                 o_cv = o_sc + align_up(16 * ns, 256), o_cc = o_cv + align_up(16 * 36 * nc, 256),
                 scene_bytes = o_cc + align_up(16 * nc, 256) + 256;
    rc = ensure(&ctx->scene_buf, &ctx->scene_cap, scene_bytes);
    if (rc) return rc;
    const size_t px = (size_t)width * rows;
    const size_t out_bytes = px * (out_format == RT_FORMAT_I32X4 ? 16 : 4);
    rc = ensure(&ctx->out_buf, &ctx->out_cap, out_bytes);
    if (rc) return rc;
    char* sb = static_cast<char*>(ctx->scene_buf);
    hipStream_t st = ctx->stream;
    HIP_TRY(hipEventRecord(ctx->ev[0], st));
    if (ns) {
        HIP_TRY(hipMemcpyAsync(sb + o_so, scene->sphere_origins, 16 * ns, hipMemcpyHostToDevice, st));
        HIP_TRY(hipMemcpyAsync(sb + o_sr, scene->sphere_radius, 4 * ns, hipMemcpyHostToDevice, st));
        HIP_TRY(hipMemcpyAsync(sb + o_sc, scene->sphere_colours, 16 * ns, hipMemcpyHostToDevice, st));
    }
    if (nc) {
        HIP_TRY(hipMemcpyAsync(sb + o_cv, scene->cube_vertices, 16 * 36 * nc, hipMemcpyHostToDevice, st));
        HIP_TRY(hipMemcpyAsync(sb + o_cc, scene->cube_colours, 16 * nc, hipMemcpyHostToDevice, st));
    }
    const float* d_origins = nullptr;
    if (ray_origins) {
        // the reference uploads all W*H origins (MainState.cpp:841-855); a
        // band needs only its own rows
        const size_t ob = px * 16;
        rc = ensure(&ctx->origin_buf, &ctx->origin_cap, ob);
        if (rc) return rc;
        HIP_TRY(hipMemcpyAsync(ctx->origin_buf, ray_origins + (size_t)4 * width * row_begin, ob,
                               hipMemcpyHostToDevice, st));
        d_origins = static_cast<const float*>(ctx->origin_buf);
    }
    rt_scene dscene = *scene;
    dscene.sphere_origins = reinterpret_cast<const float*>(sb + o_so);
    dscene.sphere_radius = reinterpret_cast<const float*>(sb + o_sr);
    dscene.sphere_colours = reinterpret_cast<const float*>(sb + o_sc);
    dscene.cube_vertices = reinterpret_cast<const float*>(sb + o_cv);
    dscene.cube_colours = reinterpret_cast<const float*>(sb + o_cc);
    HIP_TRY(hipEventRecord(ctx->ev[1], st));
    int32_t used = 0;
    rc = launch(ctx, &dscene, ray_dir, d_origins, width, row_begin, row_end, out_format, path,
                ctx->out_buf, st, &used);
    if (rc) return rc;
    HIP_TRY(hipEventRecord(ctx->ev[2], st));
    HIP_TRY(hipMemcpyAsync(host_out, ctx->out_buf, out_bytes, hipMemcpyDeviceToHost, st));
    HIP_TRY(hipEventRecord(ctx->ev[3], st));
    HIP_TRY(hipStreamSynchronize(st));
    if (timing) {
        float a = 0, b = 0, c = 0;
        (void)hipEventElapsedTime(&a, ctx->ev[0], ctx->ev[1]);
        (void)hipEventElapsedTime(&b, ctx->ev[1], ctx->ev[2]);
        (void)hipEventElapsedTime(&c, ctx->ev[2], ctx->ev[3]);
        timing->upload_us = 1e3 * a;
        timing->kernel_us = 1e3 * b;
        timing->download_us = 1e3 * c;
        timing->path = used;
        timing->total_us = std::chrono::duration<double, std::micro>(
                               std::chrono::steady_clock::now() - t0).count();
    }
    return RT_OK;
}

int rt_render(rt_ctx* ctx, const rt_scene* scene, const float ray_dir[4], const float* ray_origins,
              int32_t width, int32_t height, int32_t row_begin, int32_t row_end,
              int32_t out_format, void* host_out, rt_timing* timing) {
    return rt_render_path(ctx, scene, ray_dir, ray_origins, width, height, row_begin, row_end,
                          out_format, RT_PATH_AUTO, host_out, timing);
}

int rt_render_multi(rt_ctx* const* ctxs, int32_t num_ctx, const rt_scene* scene,
                    const float ray_dir[4], const float* ray_origins, int32_t width,
                    int32_t height, int32_t row_begin, int32_t row_end, int32_t out_format,
                    void* host_out, rt_timing* timings) {
    if (!ctxs || num_ctx <= 0 || !ray_dir || !host_out) return RT_ERR_INVALID_ARG;
    for (int32_t i = 0; i < num_ctx; ++i)
        if (!ctxs[i]) return RT_ERR_INVALID_ARG;
    int rc = check_args(scene, width, height, row_begin, row_end, out_format);
    if (rc) return rc;
    // contiguous bands of whole rows, sizes differing by at most one; more
    // contexts than rows leave the surplus ones idle
    const int32_t rows = row_end - row_begin;
    const int32_t n = std::min(num_ctx, rows);
    const size_t row_bytes = (size_t)width * (out_format == RT_FORMAT_I32X4 ? 16 : 4);
    std::vector<int> status((size_t)n, RT_OK);
    auto band = [&](int32_t i) {
        const int32_t rb = row_begin + (int32_t)((int64_t)rows * i / n);
        const int32_t re = row_begin + (int32_t)((int64_t)rows * (i + 1) / n);
        char* dst = static_cast<char*>(host_out) + (size_t)(rb - row_begin) * row_bytes;
        status[(size_t)i] = rt_render(ctxs[i], scene, ray_dir, ray_origins, width, height, rb,
                                      re, out_format, dst, timings ? &timings[i] : nullptr);
    };
    if (n == 1) {
        band(0);
    } else {
        std::vector<std::thread> workers;
        workers.reserve((size_t)n);
        for (int32_t i = 0; i < n; ++i) workers.emplace_back(band, i);
        for (auto& w : workers) w.join();
    }
    for (int32_t i = n; timings && i < num_ctx; ++i) timings[i] = rt_timing{};
    for (int s : status)
        if (s != RT_OK) return s;
    return RT_OK;
}

int rt_render_device(rt_ctx* ctx, const rt_scene* device_scene, const float ray_dir[4],
                     const float* device_ray_origins, int32_t width, int32_t height,
                     int32_t row_begin, int32_t row_end, int32_t out_format, int32_t path,
                     void* device_out, void* stream) {
    if (!ctx || !ray_dir || !device_out) return RT_ERR_INVALID_ARG;
    int rc = check_args(device_scene, width, height, row_begin, row_end, out_format);
    if (rc) return rc;
    if (path < RT_PATH_AUTO || path > RT_PATH_GENERIC) return RT_ERR_INVALID_ARG;
    HIP_TRY(hipSetDevice(ctx->device));
    hipStream_t st = stream ? static_cast<hipStream_t>(stream) : ctx->stream;
    // launch() reads origins from the band's first row
    const float* band_origins =
        device_ray_origins ? device_ray_origins + (size_t)4 * width * row_begin : nullptr;
    return launch(ctx, device_scene, ray_dir, band_origins, width, row_begin, row_end,
                  out_format, path, device_out, st, nullptr);
}

int rt_host_register(void* host_ptr, int64_t bytes) {
    if (!host_ptr || bytes <= 0) return RT_ERR_INVALID_ARG;
    HIP_TRY(hipHostRegister(host_ptr, (size_t)bytes, hipHostRegisterPortable));
    return RT_OK;
}

int rt_host_unregister(void* host_ptr) {
    if (!host_ptr) return RT_ERR_INVALID_ARG;
    HIP_TRY(hipHostUnregister(host_ptr));
    return RT_OK;
}

int rt_shared_alloc(rt_ctx* ctx, int64_t bytes, void** device_ptr, rt_ipc_handle* handle) {
    if (!ctx || bytes <= 0 || !device_ptr || !handle) return RT_ERR_INVALID_ARG;
    static_assert(sizeof(hipIpcMemHandle_t) == sizeof(rt_ipc_handle), "IPC handle size");
    *device_ptr = nullptr;
    HIP_TRY(hipSetDevice(ctx->device));
    void* p = nullptr;
    // its own allocation: an IPC handle names a whole hipMalloc block
    if (hipMalloc(&p, (size_t)bytes) != hipSuccess) return RT_ERR_OUT_OF_MEMORY;
    hipIpcMemHandle_t h;
    if (hipIpcGetMemHandle(&h, p) != hipSuccess) {
        (void)hipFree(p);
        return RT_ERR_HIP;
    }
    std::memcpy(handle->bytes, &h, sizeof h);
    *device_ptr = p;
    return RT_OK;
}

int rt_shared_open(rt_ctx* ctx, const rt_ipc_handle* handle, void** device_ptr) {
    if (!ctx || !handle || !device_ptr) return RT_ERR_INVALID_ARG;
    *device_ptr = nullptr;
    HIP_TRY(hipSetDevice(ctx->device));
    hipIpcMemHandle_t h;
    std::memcpy(&h, handle->bytes, sizeof h);
    // mapped for this context's device (peer access over xGMI when the
    // allocation lives on another GPU)
    HIP_TRY(hipIpcOpenMemHandle(device_ptr, h, hipIpcMemLazyEnablePeerAccess));
    return RT_OK;
}

int rt_shared_close(rt_ctx* ctx, void* device_ptr) {
    if (!ctx || !device_ptr) return RT_ERR_INVALID_ARG;
    HIP_TRY(hipSetDevice(ctx->device));
    HIP_TRY(hipIpcCloseMemHandle(device_ptr));
    return RT_OK;
}

int rt_shared_free(rt_ctx* ctx, void* device_ptr) {
    if (!ctx || !device_ptr) return RT_ERR_INVALID_ARG;
    HIP_TRY(hipSetDevice(ctx->device));
    HIP_TRY(hipDeviceSynchronize());
    HIP_TRY(hipFree(device_ptr));
    return RT_OK;
}

int rt_profile_enable(rt_ctx* ctx, int enable) {
    if (!ctx) return RT_ERR_INVALID_ARG;
    ctx->profile = enable != 0;
    return RT_OK;
}

int rt_profile_read(rt_ctx* ctx, double* prep_ms, double* bin_ms, double* trace_ms,
                    int32_t* n_renders) {
    if (!ctx) return RT_ERR_INVALID_ARG;
    HIP_TRY(hipSetDevice(ctx->device));
    double sums[3] = {0, 0, 0};
    for (size_t q = 0; q + 5 < ctx->prof_used; q += 6) {
        for (int k = 2; k >= 0; --k)  // the last kernel that ran
            if (!ctx->prof_skipped[q / 2 + k]) {
                HIP_TRY(hipEventSynchronize(ctx->prof_events[q + 2 * k + 1]));
                break;
            }
        for (int k = 0; k < 3; ++k) {
            if (ctx->prof_skipped[q / 2 + k]) continue;
            float ms = 0.0f;
            HIP_TRY(hipEventElapsedTime(&ms, ctx->prof_events[q + 2 * k],
                                        ctx->prof_events[q + 2 * k + 1]));
            sums[k] += ms;
        }
    }
    if (prep_ms) *prep_ms = sums[0];
    if (bin_ms) *bin_ms = sums[1];
    if (trace_ms) *trace_ms = sums[2];
    if (n_renders) *n_renders = ctx->prof_count;
    ctx->prof_used = 0;  // the events stay in the pool
    ctx->prof_count = 0;
    return RT_OK;
}

int rt_device_info(rt_ctx* ctx, char* name, int32_t name_len, int32_t* n_cu, int64_t* total_mem) {
    if (!ctx) return RT_ERR_INVALID_ARG;
    hipDeviceProp_t prop;
    HIP_TRY(hipGetDeviceProperties(&prop, ctx->device));
    if (name && name_len > 0) {
        std::snprintf(name, (size_t)name_len, "%s (%s)", prop.name, prop.gcnArchName);
    }
    if (n_cu) *n_cu = prop.multiProcessorCount;
    if (total_mem) *total_mem = (int64_t)prop.totalGlobalMem;
    return RT_OK;
}

// Test hooks (not part of the reference interface).
int rt_selftest_fp32(rt_ctx* ctx, const float* host_in, int32_t n, float* host_sqrt,
                     float* host_div) {
    if (!ctx || !host_in || n <= 0 || !host_sqrt || !host_div) return RT_ERR_INVALID_ARG;
    HIP_TRY(hipSetDevice(ctx->device));
    float* d = nullptr;
    HIP_TRY(hipMalloc(&d, sizeof(float) * 3 * (size_t)n));
    HIP_TRY(hipMemcpy(d, host_in, sizeof(float) * n, hipMemcpyHostToDevice));
    fp32_selftest_kernel<<<dim3((n + 255) / 256), dim3(256), 0, ctx->stream>>>(d, n, d + n,
                                                                            d + 2 * (size_t)n);
    HIP_TRY(hipStreamSynchronize(ctx->stream));
    HIP_TRY(hipMemcpy(host_sqrt, d + n, sizeof(float) * n, hipMemcpyDeviceToHost));
    HIP_TRY(hipMemcpy(host_div, d + 2 * (size_t)n, sizeof(float) * n, hipMemcpyDeviceToHost));
    (void)hipFree(d);
    return RT_OK;
}

// Host evaluation of the prep step (same __host__ __device__ code the prep
// kernel runs), for the CPU-side culling-bound tests.  Writes the box as
// int32[4] (x0, y0, x1, y1) and returns 1 when the triangle is valid.
int rt_debug_triangle_box(const float v0[3], const float v1[3], const float v2[3],
                          const float dir[4], int32_t width, int32_t row_begin, int32_t row_end,
                          int32_t box_out[4], float cls_out[8]) {
    TriRec r{};
    Box b{};
    Cls k{};
    bool bad = false;
    const bool ok = prep_triangle(v0, v1, v2, dir[0], dir[1], dir[2], width, row_begin, row_end,
                                  &r, &b, &k, &bad);
    box_out[0] = b.x0; box_out[1] = b.y0; box_out[2] = b.x1; box_out[3] = b.y1;
    if (cls_out) std::memcpy(cls_out, &k, sizeof k);
    return ok ? 1 : 0;
}

// Diagnostics: select a trace-kernel ablation (0 = normal).
int rt_debug_set_list_budget(rt_ctx* ctx, int64_t bytes) {
    if (!ctx || bytes < 0) return RT_ERR_INVALID_ARG;
    ctx->list_budget = bytes ? bytes : (int64_t)4 << 30;
    return RT_OK;
}

int rt_debug_set_bin_masks(rt_ctx* ctx, int enable) {
    if (!ctx) return RT_ERR_INVALID_ARG;
    ctx->bin_masks = enable != 0;
    return RT_OK;
}

int rt_debug_set_coarse_cull(rt_ctx* ctx, int enable) {
    if (!ctx) return RT_ERR_INVALID_ARG;
    ctx->coarse_cull = enable < 0 ? RT_COARSE_CULL : enable;  // < 0: the default
    return RT_OK;
}

int rt_debug_set_small_path(rt_ctx* ctx, int enable) {
    if (!ctx) return RT_ERR_INVALID_ARG;
    ctx->small_path = enable != 0;
    return RT_OK;
}

int rt_debug_set_trace_mode(rt_ctx* ctx, int mode) {
    if (!ctx || mode < 0 || mode > 4) return RT_ERR_INVALID_ARG;
    ctx->trace_mode = mode;
    return RT_OK;
}

#if RT_TIMELINE
// Diagnostics build only: per-wave timeline buffer (8 x uint32 per wave).
int rt_debug_set_timeline(rt_ctx* ctx, void* device_buf) {
    if (!ctx) return RT_ERR_INVALID_ARG;
    HIP_TRY(hipSetDevice(ctx->device));
    HIP_TRY(hipMemcpyToSymbol(HIP_SYMBOL(g_timeline), &device_buf, sizeof(void*)));
    return RT_OK;
}
#endif

int rt_debug_tile_shape(int32_t* w, int32_t* h) {
    if (!w || !h) return RT_ERR_INVALID_ARG;
    *w = kWaveTile;
    *h = kWaveTileH;
    return RT_OK;
}

int rt_debug_block_shape(int32_t* w, int32_t* h) {
    if (!w || !h) return RT_ERR_INVALID_ARG;
    *w = kWaveTile;
    *h = kBlockH;
    return RT_OK;
}

int rt_debug_sphere_box(const float origin[4], float radius, const float dir[4], int32_t width,
                        int32_t row_begin, int32_t row_end, int32_t box_out[4],
                        float cls_out[8]) {
    SphRec r{};
    Box b{};
    Cls k{};
    bool bad = false;
    prep_sphere(origin, radius, dir[0], dir[1], dir[2], dir[3], width, row_begin, row_end, &r, &b,
                &k, &bad);
    box_out[0] = b.x0; box_out[1] = b.y0; box_out[2] = b.x1; box_out[3] = b.y1;
    if (cls_out) std::memcpy(cls_out, &k, sizeof k);
    return bad ? 0 : 1;
}

}  // extern "C"
