/*
 * rt_hip_debug.h -- test and diagnostics hooks exported by librt_hip.so.
 *
 * Not part of the drop-in boundary (rt_hip.h) and with no reference
 * counterpart: these let the test suite check the binned path's culling
 * bounds on the host, check the device's fp32 rounding, and time ablated
 * variants of the trace kernel.  A MainState integration never calls them.
 */
#ifndef RT_HIP_DEBUG_H
#define RT_HIP_DEBUG_H

#include <stdint.h>

#include "rt_hip.h"

#ifdef __cplusplus
extern "C" {
#endif

/* Device sqrtf and x / 180.0f for n inputs (both must be correctly rounded
 * for parity with the reference's SSE build, MainState.cpp:321, :400). */
int rt_selftest_fp32(rt_ctx* ctx, const float* host_in, int32_t n,
                     float* host_sqrt, float* host_div);

/* Host evaluation of the prep kernel's per-triangle / per-sphere culling
 * data (the same __host__ __device__ code): inclusive pixel box
 * (x0, y0, x1, y1) and the 8-float tile classifier.  Return 1 when the
 * primitive can report a hit at all (triangle) / has finite data (sphere). */
int rt_debug_triangle_box(const float v0[3], const float v1[3],
                          const float v2[3], const float dir[4], int32_t width,
                          int32_t row_begin, int32_t row_end,
                          int32_t box_out[4], float cls_out[8]);
int rt_debug_sphere_box(const float origin[4], float radius,
                        const float dir[4], int32_t width, int32_t row_begin,
                        int32_t row_end, int32_t box_out[4], float cls_out[8]);

/* Pixel shape of the tile one wave traces (w x h). */
int rt_debug_tile_shape(int32_t* w, int32_t* h);

/* Pixel shape of the row block the coarse kernel classifies (w x h): a tile
 * is h_tile / h blocks stacked vertically, block j holding lane row j of
 * every lane, so each block's verdict (skip / test / u,v inside) is
 * wave-uniform for that row. */
int rt_debug_block_shape(int32_t* w, int32_t* h);

/* Byte budget for the coarse candidate lists (8 B x (primitives + 16) per
 * 64x64 bin: an id and a tile word; 20 B with RT_ROWBITS=1); binned frames
 * over it render as internal row bands.
 * 0 restores the default (4 GiB). */
int rt_debug_set_list_budget(rt_ctx* ctx, int64_t bytes);

/* Coarse binning source: 1 (default) = the separable bin-row / bin-column
 * masks prep publishes, 0 = scan every primitive's box (the path frames with
 * more than 4096 bin rows + columns take). */
int rt_debug_set_bin_masks(rt_ctx* ctx, int enable);

/* Scenes of at most 512 primitives: 1 (default) = trace_small_kernel (each
 * tile wave classifies its candidates itself, no coarse kernel), 0 = the
 * general prep -> coarse -> trace path. */
int rt_debug_set_small_path(rt_ctx* ctx, int enable);
/* Scenes of at most 128 primitives: 1 (default) = frame_small_kernel (prep,
 * classification and trace in one kernel, records in LDS) on frames whose
 * grid is resident at once, 2 = on every frame size (tests), 0 = prep_kernel
 * + trace_small_kernel (A/B and tests).  Needs the small path (above). */
int rt_debug_set_small_fused(rt_ctx* ctx, int enable);

/* Waves per wave tile in the binned trace: 0 (default) = by frame size
 * (trace3_split_kernel, 4 / 2 waves per tile, on frames of at most 2048 /
 * 4096 wave tiles), 1 = always one (trace3_kernel), 2 or 4 = always that
 * many. */
int rt_debug_set_trace_split(rt_ctx* ctx, int waves);

/* Waves per coarse bin (coarse3_kernel): 0 (default) = by band size (8 up to
 * 256 bins, 4 up to 1024, then 1), or always 1, 2, 4 or 8. */
int rt_debug_set_coarse_waves(rt_ctx* ctx, int waves);

/* Binned frames without the coarse kernel (trace_bin_kernel: every wave tile
 * ANDs its bin's mask words and classifies the candidates itself; scenes of
 * at most 1024 primitives): 0 (default) = automatic (frames above 4096 wave
 * tiles whose previous binned frame on this context had a box overdraw below
 * 4 frames for int32x4, 1 for RGBA8), 1 = wherever it applies, 2 = never. */
int rt_debug_set_trace_bin(rt_ctx* ctx, int mode);

/* How the overdraw verdict behind the automatic path choice reaches the
 * host: 0 (default where the device can map the context's page-locked word)
 * = the coarse kernel / trace_bin_kernel store it there themselves, every
 * binned launch; 1 = they store it in device memory and a 4-byte copy every
 * 8th binned launch brings it over (the library's fallback, and round 5's
 * only way).  RT_ERR_UNSUPPORTED for 0 where the word is not mapped. */
int rt_debug_set_verdict_copy(rt_ctx* ctx, int copy);

/* The box overdraw of the last binned render of >= 1 band on this context
 * (prep's sum of the primitives' pixel-box areas over the band's area, in
 * frames; what the automatic path choices gate on).  Synchronises the
 * device.  0 before any such render. */
int rt_debug_last_overdraw(rt_ctx* ctx, double* frames);
/* Coarse depth cull of sphere candidates in coarse bins with at least
 * `enable` sphere candidates (1 = every bin, 0 = off: every candidate the tile
 * classifier keeps stays; negative = the build's default; A/B and tests). */
int rt_debug_set_coarse_cull(rt_ctx* ctx, int enable);
/* Triangles join the coarse depth cull in bins whose wave tiles keep at
 * least this many candidates on average (0 = never, negative = the build's
 * defaults: 4 for int32x4 renders, 2 for RGBA8 renders; a value >= 0 applies
 * to both formats). */
int rt_debug_set_coarse_cull_tri(rt_ctx* ctx, int min_candidates);
/* ... and only in frames whose primitive boxes, summed, cover the frame at
 * least `frames` times (the trace is then bound by its tests rather than its
 * stores; 0 = every frame, negative = the build's defaults: 5 for int32x4
 * renders, 0 for RGBA8 renders, whose trace is bound by its tests, and in
 * either format only in bands of at least 768 coarse bins, since fewer coarse
 * waves cannot hide the cull's latency).  A value >= 0 applies to both
 * formats and every band size. */
int rt_debug_set_coarse_cull_overdraw(rt_ctx* ctx, int frames);
/* The bounds tri_t_bounds gives the trace's computed fp64 t over pixels
 * [xa, xb] x [ya, yb] (host evaluation; returns 0 without a bound). */
int rt_debug_triangle_t_bounds(const float v0[3], const float v1[3], const float v2[3],
                               const float dir[4], int32_t width, int32_t row_begin,
                               int32_t row_end, int32_t xa, int32_t xb, int32_t ya, int32_t yb,
                               double out[2]);
/* Wave-tile build used by the binned path: 0 = by frame size (128x2 tiles
 * for frames of >= 512 MiB, else 16x16), 1 = 16x16, 2 = 128x2. */
int rt_debug_set_tile_variant(rt_ctx* ctx, int variant);
/* The wide (128x2) build's triangle prep and tile shape (host culling tests). */
int rt_debug_triangle_box_wide(const float v0[3], const float v1[3], const float v2[3],
                               const float dir[4], int32_t width, int32_t row_begin,
                               int32_t row_end, int32_t box_out[4], float cls_out[8]);
int rt_debug_tile_shape_wide(int32_t* w, int32_t* h);

/* Host evaluation of the device's restatement of glibc 2.35 sinf / cosf
 * (the same __host__ __device__ code rt_cube_build_device runs), for the
 * CPU test against the host's libm. */
int rt_debug_glibc_sincosf(const float* x, int64_t n, float* sin_out,
                           float* cos_out);
/* The same restatement run on the device (synchronous; device pointers). */
int rt_selftest_sincosf(rt_ctx* ctx, const float* device_in, int64_t n,
                        float* device_sin, float* device_cos);

#ifdef __cplusplus
}
#endif
#endif /* RT_HIP_DEBUG_H */
