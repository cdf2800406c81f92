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
// The kernels and their host launch() are in rt_trace.inc, compiled here
// twice: 16x16 wave tiles (namespace tile16) and 128x2 tiles (namespace
// wide, frames of >= 512 MiB, whose stores drain faster from 2-KiB row
// segments).
// This file holds the context, the dispatcher and the C ABI.
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
#include <mutex>
#include <thread>
#include <vector>

#include "rt_args.h"
#include "rt_hip.h"
#include "rt_hip_debug.h"
#include "rt_hip_diag.h"
#include "rt_internal.h"

#pragma clang fp contract(off)

// Diagnostics build (make RT_DIAG=1): the trace-kernel ablations of
// rt_debug_set_trace_mode (rt_hip_diag.h) and the RT_TIMELINE / RT_SKIP_DIAG
// instrumentation.  The default library instantiates and exports none of it.
#ifndef RT_DIAG
#define RT_DIAG 0
#endif
#if !RT_DIAG && ((defined(RT_TIMELINE) && RT_TIMELINE) || (defined(RT_SKIP_DIAG) && RT_SKIP_DIAG))
#error "RT_TIMELINE and RT_SKIP_DIAG are diagnostics: build with RT_DIAG=1"
#endif

#ifndef RT_BIN_MASKS
#define RT_BIN_MASKS 1            // default of rt_debug_set_bin_masks
#endif
#ifndef RT_COARSE_CULL
#define RT_COARSE_CULL 10  // default of rt_debug_set_coarse_cull: bins with >= 10 sphere candidates
#endif
#ifndef RT_COARSE_CULL_TRI
#define RT_COARSE_CULL_TRI 4  // default of rt_debug_set_coarse_cull_tri: triangles join the cull
                              // in bins whose tiles keep >= this many candidates on average
#endif
#ifndef RT_SMALL_FUSED
#define RT_SMALL_FUSED 1  // default of rt_debug_set_small_fused
#endif
#ifndef RT_COARSE_CULL_OVERDRAW
#define RT_COARSE_CULL_OVERDRAW 5  // default of rt_debug_set_coarse_cull_overdraw: ... in frames
                                   // whose primitive boxes cover the frame >= 5 times
#endif
#ifndef RT_COARSE_CULL_TRI_RGBA8
#define RT_COARSE_CULL_TRI_RGBA8 2  // the triangle threshold for Texture (RGBA8) renders
#endif
#ifndef RT_COARSE_CULL_OVERDRAW_RGBA8
#define RT_COARSE_CULL_OVERDRAW_RGBA8 0  // the same gate for Texture (RGBA8) renders: every
                                         // frame (its trace is bound by its tests, not by
                                         // its stores)
#endif
#ifndef RT_SPLIT4_TILES
#define RT_SPLIT4_TILES 2048  // trace3_split_kernel with 4 waves per tile up to this many tiles
#endif
#ifndef RT_SPLIT2_TILES
#define RT_SPLIT2_TILES 4096  // ... with 2 waves per tile up to this many (round 4: at
                              // 8160, 1920x1080, flat; 4 waves win below 2048 tiles,
                              // 2 up to 4096, one above)
#endif
#ifndef RT_COARSE_W8_BINS
#define RT_COARSE_W8_BINS 256  // coarse3_kernel with 8 waves per bin in bands up to this many
                               // bins (round 4: 80 and 240 bins 0.3-2.3 us faster than 4)
#endif
#ifndef RT_COARSE_W4_BINS
#define RT_COARSE_W4_BINS 1024  // coarse3_kernel with 4 waves per bin in bands up to this many
                                // bins (round 4: 4 waves fastest from 80 to 920 bins, one
                                // at 4096 and up)
#endif
#ifndef RT_COARSE_W2_BINS
#define RT_COARSE_W2_BINS 1024  // ... with 2 waves per bin up to this many (none by default)
#endif
#ifndef RT_TRACE_BIN_OD10
#define RT_TRACE_BIN_OD10 40  // trace_bin_kernel (auto) for int32x4 frames below this box overdraw,
                              // in tenths of a frame (round 5, one stream, config 3's scene scaled:
                              // overdraw 0.08 / 0.3 / 0.7 / 1.4 / 2.8 / 4.3 / 6.1 frames, coarse path
                              // 55.0 / 56.0 / 55.5 / 55.8 / 57.4 / 60.0 / 61.5 us per frame, no coarse
                              // 51.3 / 51.3 / 49.6 / 49.8 / 53.9 / 60.9 / 69.2)
#endif
#ifndef RT_TRACE_BIN_OD10_RGBA8
#define RT_TRACE_BIN_OD10_RGBA8 10  // ... for RGBA8 frames (same scenes: coarse path 37.5 / 39.3 /
                                    // 40.2 / 42.0 / 44.5 / 46.7 / 47.9, no coarse 29.9 / 31.6 / 34.3 /
                                    // 40.0 / 49.3 / 58.1 / 65.9; with 3 frames in flight at overdraw
                                    // 0.08 / 1.4 / 2.8: coarse 18.3 / 27.5 / 32.5, no coarse 17.3 /
                                    // 30.6 / 40.6, so 1 frame, not the one-stream crossover)
#endif
#ifndef RT_VERDICT_DIRECT
#define RT_VERDICT_DIRECT 1  // the kernels write the overdraw verdict into the host word themselves
                             // (every binned launch, no copy; rt_ctx::od_verdict)
#endif
#ifndef RT_COARSE_CULL_TRI_BINS
#define RT_COARSE_CULL_TRI_BINS 768  // triangles join the cull only in bands of at least this
                                     // many coarse bins: fewer coarse waves run as one
                                     // generation and cannot hide the cull's latency (round 4:
                                     // 640x480 to 1920x1080 frames 1-27 us slower with it at
                                     // box overdraw 5-20, 2560x1440 up to 16 us faster;
                                     // DESIGN.md §3.5)
#endif

// ===========================================================================
// Host side
// ===========================================================================
struct rt_ctx {
    int device = 0;
    hipStream_t stream = nullptr;
    // workspace (grow-only)
    void* scene_buf = nullptr;  size_t scene_cap = 0;   // host-API scene copy
    void* scene_stage = nullptr; size_t stage_cap = 0;  // its page-locked host staging
    void* origin_buf = nullptr; size_t origin_cap = 0;  // host-API explicit origins
    void* out_buf = nullptr;    size_t out_cap = 0;     // host-API frame
    void* rec_buf = nullptr;    size_t rec_cap = 0;     // TriRec/SphRec/boxes/flag
    void* list_buf = nullptr;   size_t list_cap = 0;    // coarse-bin candidate lists
    unsigned* flag = nullptr;   // non-finite scene flag (generation-stamped)
    // a recent binned frame's overdraw verdict (0 = none yet, 1 = below
    // RT_TRACE_BIN_OD10_RGBA8 tenths of a frame, 2 = below RT_TRACE_BIN_OD10,
    // 3 = above): the coarse or self-binning trace kernel writes it straight
    // into this page-locked, device-mapped word (od_verdict_dev, a
    // system-scope store, every binned launch: RT_VERDICT_DIRECT), or, where
    // that mapping is unavailable, to flag word 6 (device memory), which
    // every 8th binned launch copies asynchronously into the word.  The word
    // picks the next frame's path (performance only; both paths are exact).
    // Its lifetime is the context's: allocated in rt_init, freed only in
    // rt_destroy after every write into it has landed.
    unsigned* od_verdict = nullptr;
    unsigned* od_verdict_dev = nullptr;  // its device mapping (direct writes), or null
    unsigned* od_verdict_map = nullptr;  // the mapping, kept (rt_debug_set_verdict_copy)
    unsigned verdict_copies = 0;  // copies enqueued
    // recorded behind every verdict copy: rt_destroy waits for the last one
    // only (a context's renders move to another stream only after a
    // synchronisation, rt_hip.h, so the last copy is the only one in flight)
    hipEvent_t verdict_done = nullptr;
    // rt_render: the verdict copy waits until after the frame download, so
    // download_us times the frame alone (launch() sets verdict_due instead)
    bool defer_verdict = false;
    bool verdict_due = false;
    unsigned gen = 0;
    unsigned od_launches = 0;  // binned launches: picks the box-overdraw slot
    unsigned long long od_area = 0;  // the last such launch's area, 64-pixel units
    int trace_mode = 0;  // diagnostics ablation (RT_DIAG builds), see trace3_kernel
    int last_kernel = RT_KERNEL_NONE;  // the dominant kernel of the last launch (rt_last_kernel)
    int tile_variant = 0;  // 0 = by frame size, 1 = 16x16 tiles, 2 = the wide (128x2) tiles
    // coarse lists take 4 B x kListStride x (primitives + 16) per 64x64 bin; a frame whose
    // lists would exceed this is rendered as internal row bands
    int64_t list_budget = (int64_t)4 << 30;
    bool bin_masks = RT_BIN_MASKS != 0;  // separable bin masks (false: coarse scans every box)
    bool small_path = true;  // <= 64 x RT_SMALL_CHUNKS primitives: trace_small_kernel
    // <= 64 x RT_FUSED_CHUNKS primitives on frames whose grid is resident at
    // once: frame_small_kernel (1; 2 = on every frame size, tests; 0 = off)
    int small_fused = RT_SMALL_FUSED;
    // waves per wave tile in the binned trace: 0 = by frame size
    // (trace3_split_kernel on small frames), 1 = one (trace3_kernel), 2 / 4
    int trace_split = 0;
    // waves per coarse bin: 0 = by band size, 1 / 2 / 4 / 8
    int coarse_waves = 0;
    // binned frames without the coarse kernel (trace_bin_kernel): 0 = auto
    // (frames above the split sizes whose last binned frame had a box
    // overdraw below the format's threshold), 1 = always where it applies,
    // 2 = never
    int trace_bin = 0;
    int n_cu = 256;  // compute units (rt_init)
    // coarse depth cull of sphere candidates in bins with at least this many
    // candidates (0 = off)
    int coarse_cull = RT_COARSE_CULL;
    // triangles join the depth cull in bins whose tiles keep at least this
    // many candidates on average (0 = never)
    int coarse_cull_tri = RT_COARSE_CULL_TRI;
    int coarse_cull_tri_rgba8 = RT_COARSE_CULL_TRI_RGBA8;  // (RGBA8 renders)
    // ... in frames whose boxes' summed area is at least this many frames
    // (int32x4 renders; RGBA8 renders take the second gate)
    unsigned coarse_cull_overdraw = RT_COARSE_CULL_OVERDRAW;
    unsigned coarse_cull_overdraw_rgba8 = RT_COARSE_CULL_OVERDRAW_RGBA8;
    // ... in bands of at least this many coarse bins
    int64_t coarse_cull_tri_bins = RT_COARSE_CULL_TRI_BINS;
    hipEvent_t ev[4] = {nullptr, nullptr, nullptr, nullptr};
    // rt_render's kernel span: ev[1] / ev[2] ride on the first / last kernel
    // of the render (set only while rt_render_path enqueues it)
    hipEvent_t span_start = nullptr, span_stop = nullptr;
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
hipStream_t ctx_stream(rt_ctx* ctx) {
    if (!ctx->stream && hipStreamCreateWithFlags(&ctx->stream, hipStreamNonBlocking) != hipSuccess)
        ctx->stream = nullptr;
    return ctx->stream;
}
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

using rt_args::check_args;

struct KEv {
    hipEvent_t start, stop;
};

#define HIP_TRY(x)                                    \
    do {                                              \
        if ((x) != hipSuccess) return RT_ERR_HIP;     \
    } while (0)

// Launch `kernel` on `stream`; with events, through hipExtLaunchKernelGGL so
// the start / stop timestamps are the kernel's own (no extra queue packets
// between the kernels).  Either event may be null.
template <typename K, typename... A>
int launch_k(K kernel, dim3 grid, dim3 block, hipStream_t stream, KEv ev, A... args) {
    if (ev.start || ev.stop)
        hipExtLaunchKernelGGL(kernel, grid, block, 0, stream, ev.start, ev.stop, 0, args...);
    else
        kernel<<<grid, block, 0, stream>>>(args...);
    return hipGetLastError() == hipSuccess ? RT_OK : RT_ERR_HIP;
}

// The events one kernel of a render carries: its profiling pair (`pe`,
// rt_profile_enable), else the render's span -- rt_render's kernel_us is
// the first kernel's start to the last kernel's end, the kernels' own
// timestamps, so host enqueue gaps in front of them are not kernel time.
// The span's start is taken once (the first kernel of the first band).
KEv kernel_events(rt_ctx* ctx, const hipEvent_t* pe, bool first, bool last) {
    if (pe) return KEv{pe[0], pe[1]};
    KEv e{nullptr, last ? ctx->span_stop : nullptr};
    if (first) {
        e.start = ctx->span_start;
        ctx->span_start = nullptr;
    }
    return e;
}

// A profiled kernel slot that runs nothing: flagged, so it reads 0 ms.
// (Recording the two events back to back would time the marker packets
// themselves, ~5 us, not a kernel.)
int skip_k(rt_ctx* ctx, const hipEvent_t* ev) {
    if (!ev) return RT_OK;
    ctx->prof_skipped[(size_t)(ev - ctx->prof_events.data()) / 2] = 1;
    return RT_OK;
}

// The overdraw verdict (flag word 6) into the context's page-locked word: a
// 4-byte copy behind the frame's kernels on `stream`, then the context's
// event, which rt_destroy waits for.
int enqueue_verdict_copy(rt_ctx* ctx, hipStream_t stream) {
    HIP_TRY(hipMemcpyAsync(ctx->od_verdict, ctx->flag + 6, sizeof(unsigned),
                           hipMemcpyDeviceToHost, stream));
    ++ctx->verdict_copies;
    HIP_TRY(hipEventRecord(ctx->verdict_done, stream));
    return RT_OK;
}

}  // namespace

// The kernels and launch(), once per wave-tile shape (rt_trace.inc).
// 16x16 tiles suit frames below 512 MiB; larger frames store faster from
// 128x2 tiles (a lane's 4 pixels: 2 along x, 64 apart, in 2 rows; DESIGN.md
// §3.5: 64x4 and 256x1 measured slower on configs 4 and 5).
#ifndef RT_TILE_NARROW
#define RT_TILE_NARROW 16
#endif
#ifndef RT_TILE_WIDE
#define RT_TILE_WIDE 128
#endif
// nontemporal frame stores per build: bit 0 int32x4, bit 1 RGBA8
#ifndef RT_NT_NARROW
#define RT_NT_NARROW 2  // the 16x16 build: RGBA8 only (int32x4 measured much slower)
#endif
#ifndef RT_NT_WIDE
#define RT_NT_WIDE 3
#endif
#ifndef RT_ROWS_NARROW
#define RT_ROWS_NARROW 4  // pixels per lane in the 16x16 build (A/B variants: 8 = 16x32 tiles)
#endif
#define RT_TILE_W RT_TILE_NARROW
#define RT_NT_STORES RT_NT_NARROW
#define RT_ROWS RT_ROWS_NARROW
namespace tile16 {
#include "rt_trace.inc"
}  // namespace tile16
#undef RT_TILE_W
#undef RT_NT_STORES
#undef RT_ROWS
#define RT_TILE_W RT_TILE_WIDE
#define RT_NT_STORES RT_NT_WIDE
namespace wide {
#include "rt_trace.inc"
}  // namespace wide
#undef RT_TILE_W

namespace {

// fp32 self-test: the device's sqrtf and '/' must be correctly rounded.
__global__ void fp32_selftest_kernel(const float* in, int n, float* out_sqrt, float* out_div) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    out_sqrt[i] = sqrtf(in[i]);
    out_div[i] = in[i] / 180.0f;
}

// Are the explicit ray origins of rows [row_begin, row_begin + n / width)
// exactly the reference's implicit grid (x, y, 0, 1) (MainState.cpp:44-50)?
// Bitwise comparison; any other value sets *flag (one atomic per wave).
// `origins` starts at the band's first row.
__global__ void __launch_bounds__(256) grid_check_kernel(const float4* __restrict__ origins,
                                                         int width, int row_begin, int64_t n,
                                                         unsigned* __restrict__ flag) {
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    bool off = false;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        const float4 o = origins[i];
        const int x = (int)(i % width), y = row_begin + (int)(i / width);
        off |= __float_as_uint(o.x) != __float_as_uint((float)x) ||
               __float_as_uint(o.y) != __float_as_uint((float)y) || __float_as_uint(o.z) != 0u ||
               __float_as_uint(o.w) != __float_as_uint(1.0f);
    }
    if (__ballot(off) != 0ull && (threadIdx.x & 63) == 0) atomicOr(flag, 1u);
}

// Frames of at least this many bytes take the wide tiles (auto selection):
// 512 MiB frames store faster from wide tiles in both formats (config 5's
// 8-rank band, config 4's half frame, a 512 MiB Texture; measured with 64x4
// tiles), 384 MiB and smaller ones from 16x16.
constexpr int64_t kWideTileBytes = (int64_t)1 << 29;

// rt_debug_set_tile_variant: 0 = by frame size, 1 = 16x16, 2 = wide (128x2)
bool use_wide_tiles(const rt_ctx* ctx, int32_t width, int32_t rows, int32_t fmt) {
    const int64_t bytes = (int64_t)width * rows * (fmt == RT_FORMAT_I32X4 ? 16 : 4);
    return ctx->tile_variant == 2 || (ctx->tile_variant == 0 && bytes >= kWideTileBytes);
}

int render_launch(rt_ctx* ctx, const rt_scene* s, const float d[4], const float* origins,
                  int32_t width, int32_t row_begin, int32_t row_end, int32_t fmt, int32_t path,
                  void* out, hipStream_t stream, int32_t* used_path) {
    return use_wide_tiles(ctx, width, row_end - row_begin, fmt)
               ? wide::launch(ctx, s, d, origins, width, row_begin, row_end, fmt, path, out,
                              stream, used_path)
               : tile16::launch(ctx, s, d, origins, width, row_begin, row_end, fmt, path, out,
                                stream, used_path);
}

// The binned path's workspace for a frame of `rows` rows, in the build
// render_launch() will pick (rt_reserve; rt_render before its first event).
int reserve_launch(rt_ctx* ctx, int32_t width, int32_t rows, int32_t ns, int32_t nc,
                   int32_t fmt) {
    return use_wide_tiles(ctx, width, rows, fmt) ? wide::reserve(ctx, ns, nc, width, rows)
                                                 : tile16::reserve(ctx, ns, nc, width, rows);
}

// rt_render's own buffers: the scene copy and the frame it downloads from.
int reserve_host(rt_ctx* ctx, int32_t width, int32_t rows, int32_t ns, int32_t nc,
                 int32_t fmt) {
    const size_t scene_bytes = rt_args::scene_layout(ns, nc).bytes;
    int rc = ensure(&ctx->scene_buf, &ctx->scene_cap, scene_bytes);
    if (rc) return rc;
    // the scene is packed into page-locked staging on the host and uploaded
    // by one DMA copy, instead of five small pageable copies (grow-only)
    if (scene_bytes > ctx->stage_cap) {
        if (ctx->scene_stage) (void)hipHostFree(ctx->scene_stage);
        ctx->scene_stage = nullptr;
        ctx->stage_cap = 0;
        const size_t n = align_up(scene_bytes + scene_bytes / 4, 1 << 16);
        if (hipHostMalloc(&ctx->scene_stage, n, hipHostMallocDefault) != hipSuccess) {
            ctx->scene_stage = nullptr;
            return RT_ERR_OUT_OF_MEMORY;
        }
        ctx->stage_cap = n;
    }
    return ensure(&ctx->out_buf, &ctx->out_cap, rt_args::frame_bytes(width, rows, fmt));
}

// The HIP runtime sets up its pageable-copy staging on a process's first
// pageable transfer (7-10 ms measured inside the first rt_render's
// download).  Once per device and process, rt_init runs one
// small pageable upload and download on a temporary stream, so that this
// one-time cost is openCLInit's, not the first trace's.
int warm_transfers(int device) {
    static std::mutex mu;
    static std::vector<int> done;
    std::lock_guard<std::mutex> lock(mu);
    if ((int)done.size() <= device) done.resize((size_t)device + 1, 0);
    if (done[(size_t)device]) return RT_OK;
    hipStream_t st = nullptr;
    void* d = nullptr;
    std::vector<unsigned char> h((size_t)64 << 10);
    int rc = RT_ERR_HIP;
    if (hipStreamCreateWithFlags(&st, hipStreamNonBlocking) == hipSuccess &&
        hipMalloc(&d, h.size()) == hipSuccess &&
        hipMemcpyAsync(d, h.data(), h.size(), hipMemcpyHostToDevice, st) == hipSuccess &&
        hipMemcpyAsync(h.data(), d, h.size(), hipMemcpyDeviceToHost, st) == hipSuccess &&
        hipStreamSynchronize(st) == hipSuccess)
        rc = RT_OK;
    if (d) (void)hipFree(d);
    if (st) (void)hipStreamDestroy(st);
    if (rc == RT_OK) done[(size_t)device] = 1;
    return rc;
}

// the host-side restatements the debug hooks expose are the 16x16 build's
using namespace tile16;

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
    if (hipDeviceGetAttribute(&ctx->n_cu, hipDeviceAttributeMultiprocessorCount,
                              device_ordinal) != hipSuccess || ctx->n_cu <= 0)
        ctx->n_cu = 256;
    // (the context's own stream is created on first use, rt_internal::ctx_stream:
    // every stream takes one of the device's few hardware queues, and the
    // device API mostly runs on the caller's streams)
    for (auto& e : ctx->ev) {
        if (hipEventCreate(&e) != hipSuccess) {
            rt_destroy(ctx);
            return RT_ERR_HIP;
        }
    }
    if (hipEventCreateWithFlags(&ctx->verdict_done, hipEventDisableTiming) != hipSuccess) {
        rt_destroy(ctx);
        return RT_ERR_HIP;
    }
    // [0] non-finite flag, [1] explicit-origin grid check, [2..5] two
    // 64-bit box-overdraw slots, [6] the overdraw verdict (see launch())
    if (hipMalloc(&ctx->flag, 8 * sizeof(unsigned)) != hipSuccess ||
        hipMemset(ctx->flag, 0, 8 * sizeof(unsigned)) != hipSuccess) {
        rt_destroy(ctx);
        return RT_ERR_OUT_OF_MEMORY;
    }
    // (best effort: without it the automatic path choice keeps the coarse
    // kernel; without the coherent device mapping the verdict is copied)
    if (hipHostMalloc(reinterpret_cast<void**>(&ctx->od_verdict), 64,
                      RT_VERDICT_DIRECT ? hipHostMallocMapped | hipHostMallocCoherent
                                        : hipHostMallocDefault) == hipSuccess) {
        *ctx->od_verdict = 0u;
        void* dev = nullptr;
        if (RT_VERDICT_DIRECT &&
            hipHostGetDevicePointer(&dev, ctx->od_verdict, 0) == hipSuccess && dev)
            ctx->od_verdict_dev = ctx->od_verdict_map = static_cast<unsigned*>(dev);
    } else {
        ctx->od_verdict = nullptr;
    }
    (void)hipGetLastError();
    // One-time setup here, as openCLInit builds the program before any trace
    // (MainState.cpp:1290-1320, outside the per-trace timer :662-894): every
    // kernel's code object is loaded onto the device now, not inside the
    // first render, and the runtime's transfer staging is set up.
    hipFuncAttributes fa;
    if (tile16::preload() != RT_OK || wide::preload() != RT_OK ||
        rt_internal::preload_scene_kernels() != RT_OK ||
        hipFuncGetAttributes(&fa, reinterpret_cast<const void*>(grid_check_kernel)) !=
            hipSuccess) {
        rt_destroy(ctx);
        return RT_ERR_HIP;
    }
    // best effort: a failure here only leaves the setup to the first render
    (void)warm_transfers(device_ordinal);
    (void)hipGetLastError();
    *out_ctx = ctx;
    return RT_OK;
}

int rt_reserve(rt_ctx* ctx, int32_t width, int32_t rows, int32_t num_spheres, int32_t num_cubes,
               int32_t out_format) {
    if (!ctx || rt_args::check_reserve(width, rows, num_spheres, num_cubes, out_format))
        return RT_ERR_INVALID_ARG;
    HIP_TRY(hipSetDevice(ctx->device));
    int rc = reserve_host(ctx, width, rows, num_spheres, num_cubes, out_format);
    if (rc) return rc;
    rc = reserve_launch(ctx, width, rows, num_spheres, num_cubes, out_format);
    if (rc) return rc;
    // The host API's stream, and one small pageable upload and download on
    // it (its hardware queue's first transfers).
    hipStream_t st = rt_internal::ctx_stream(ctx);
    if (!st) return RT_ERR_HIP;
    std::vector<unsigned char> tmp(std::min<size_t>(ctx->out_cap, (size_t)64 << 10));
    HIP_TRY(hipMemcpyAsync(ctx->out_buf, tmp.data(), tmp.size(), hipMemcpyHostToDevice, st));
    HIP_TRY(hipMemcpyAsync(tmp.data(), ctx->out_buf, tmp.size(), hipMemcpyDeviceToHost, st));
    HIP_TRY(hipStreamSynchronize(st));
    return RT_OK;
}

int rt_last_kernel(rt_ctx* ctx, int32_t* kernel) {
    if (!ctx || !kernel) return RT_ERR_INVALID_ARG;
    *kernel = ctx->last_kernel;
    return RT_OK;
}

void rt_destroy(rt_ctx* ctx) {
    if (!ctx) return;
    (void)hipSetDevice(ctx->device);
    if (ctx->stream) (void)hipStreamSynchronize(ctx->stream);
    // the verdict copies of rt_render_device run on the caller's streams:
    // none may still be landing in the word (or reading flag) when it goes.
    // The context's event follows the last one; waiting for it (not for the
    // whole device) leaves other contexts' and other libraries' streams alone.
    // (Direct verdict writes come from the frames' own kernels: hipHostFree
    // below synchronises the device before it frees the word, as the HIP
    // API documents, so no kernel still writes into it.)
    if (ctx->verdict_copies && ctx->verdict_done) (void)hipEventSynchronize(ctx->verdict_done);
    if (ctx->scene_stage) (void)hipHostFree(ctx->scene_stage);
    if (ctx->od_verdict) (void)hipHostFree(ctx->od_verdict);
    ctx->od_verdict = nullptr;
    ctx->od_verdict_dev = ctx->od_verdict_map = nullptr;
    for (void* p : {ctx->scene_buf, ctx->origin_buf, ctx->out_buf, ctx->rec_buf, ctx->list_buf,
                    static_cast<void*>(ctx->flag)})
        if (p) (void)hipFree(p);
    for (auto& e : ctx->ev)
        if (e) (void)hipEventDestroy(e);
    if (ctx->verdict_done) (void)hipEventDestroy(ctx->verdict_done);
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
    // and the frame; then the binned path's workspace, all before the first
    // event, so that kernel_us times kernels and never an allocation (the
    // buffers only grow: a steady-state render allocates nothing)
    const rt_args::SceneLayout lay = rt_args::scene_layout(scene->num_spheres, scene->num_cubes);
    rc = reserve_host(ctx, width, rows, scene->num_spheres, scene->num_cubes, out_format);
    if (rc) return rc;
    if (path != RT_PATH_GENERIC && binned_ok(ray_dir, nullptr)) {
        rc = reserve_launch(ctx, width, rows, scene->num_spheres, scene->num_cubes, out_format);
        if (rc) return rc;
    }
    const size_t o_so = lay.sphere_origins, o_sr = lay.sphere_radius, o_sc = lay.sphere_colours,
                 o_cv = lay.cube_vertices, o_cc = lay.cube_colours;
    const size_t px = (size_t)width * rows;
    const size_t out_bytes = rt_args::frame_bytes(width, rows, out_format);
    char* sb = static_cast<char*>(ctx->scene_buf);
    hipStream_t st = rt_internal::ctx_stream(ctx);
    if (!st) return RT_ERR_HIP;
    // the six uploads of MainState.cpp:759-838 as one: the arrays packed at
    // their device offsets in page-locked staging (the previous call's copy
    // has completed: every rt_render synchronises before it returns), then
    // one DMA copy of the whole scene
    char* stage = static_cast<char*>(ctx->scene_stage);
    if (ns) {
        std::memcpy(stage + o_so, scene->sphere_origins, 16 * ns);
        std::memcpy(stage + o_sr, scene->sphere_radius, 4 * ns);
        std::memcpy(stage + o_sc, scene->sphere_colours, 16 * ns);
    }
    if (nc) {
        std::memcpy(stage + o_cv, scene->cube_vertices, 16 * 36 * nc);
        std::memcpy(stage + o_cc, scene->cube_colours, 16 * nc);
    }
    HIP_TRY(hipEventRecord(ctx->ev[0], st));
    if (ns || nc)
        HIP_TRY(hipMemcpyAsync(sb, stage, nc ? o_cc + 16 * nc : o_sc + 16 * ns,
                               hipMemcpyHostToDevice, st));
    const float* d_origins = nullptr;
    if (ray_origins) {
        // the reference uploads all W*H origins (MainState.cpp:841-855); a
        // band needs only its own rows
        const size_t ob = px * 16;
        rc = ensure(&ctx->origin_buf, &ctx->origin_cap, ob);
        if (rc) return rc;
        HIP_TRY(hipMemcpyAsync(ctx->origin_buf, rt_args::band_origins(ray_origins, width, row_begin), ob,
                               hipMemcpyHostToDevice, st));
        d_origins = static_cast<const float*>(ctx->origin_buf);
        if (path != RT_PATH_GENERIC && binned_ok(ray_dir, nullptr)) {
            // The reference always uploads its implicit (x, y, 0, 1) grid:
            // check the origins on the device (one streaming read) and keep
            // the binned path when they are exactly that grid.
            unsigned off = 1u;
            HIP_TRY(hipMemsetAsync(ctx->flag + 1, 0, sizeof(unsigned), st));
            const int64_t blocks = std::min<int64_t>(((int64_t)px + 255) / 256, 4096);
            grid_check_kernel<<<dim3((unsigned)blocks), dim3(256), 0, st>>>(
                static_cast<const float4*>(ctx->origin_buf), width, row_begin, (int64_t)px,
                ctx->flag + 1);
            HIP_TRY(hipGetLastError());
            HIP_TRY(hipMemcpyAsync(&off, ctx->flag + 1, sizeof(unsigned), hipMemcpyDeviceToHost, st));
            HIP_TRY(hipStreamSynchronize(st));
            if (off == 0u) d_origins = nullptr;
        }
    }
    rt_scene dscene = *scene;
    dscene.sphere_origins = reinterpret_cast<const float*>(sb + o_so);
    dscene.sphere_radius = reinterpret_cast<const float*>(sb + o_sr);
    dscene.sphere_colours = reinterpret_cast<const float*>(sb + o_sc);
    dscene.cube_vertices = reinterpret_cast<const float*>(sb + o_cv);
    dscene.cube_colours = reinterpret_cast<const float*>(sb + o_cc);
    // kernel_us: the kernels' own span (their dispatch packets' timestamps);
    // with per-kernel profiling on, markers around them instead
    const bool span = !ctx->profile;
    if (span) {
        ctx->span_start = ctx->ev[1];
        ctx->span_stop = ctx->ev[2];
    } else {
        HIP_TRY(hipEventRecord(ctx->ev[1], st));
    }
    int32_t used = 0;
    ctx->defer_verdict = true;
    ctx->verdict_due = false;
    rc = render_launch(ctx, &dscene, ray_dir, d_origins, width, row_begin, row_end, out_format, path,
                ctx->out_buf, st, &used);
    ctx->defer_verdict = false;
    ctx->span_start = ctx->span_stop = nullptr;
    if (rc) return rc;
    if (!span) HIP_TRY(hipEventRecord(ctx->ev[2], st));
    HIP_TRY(hipMemcpyAsync(host_out, ctx->out_buf, out_bytes, hipMemcpyDeviceToHost, st));
    HIP_TRY(hipEventRecord(ctx->ev[3], st));
    // the verdict copy after the frame's (download_us is the frame copy alone)
    if (ctx->verdict_due) {
        ctx->verdict_due = false;
        rc = enqueue_verdict_copy(ctx, st);
        if (rc) return rc;
    }
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
    hipStream_t st = stream ? static_cast<hipStream_t>(stream) : rt_internal::ctx_stream(ctx);
    if (!st) return RT_ERR_HIP;
    // launch() reads origins from the band's first row
    const float* band_origins = rt_args::band_origins(device_ray_origins, width, row_begin);
    return render_launch(ctx, device_scene, ray_dir, band_origins, width, row_begin, row_end,
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
    hipStream_t st = rt_internal::ctx_stream(ctx);
    if (!st) {
        (void)hipFree(d);
        return RT_ERR_HIP;
    }
    fp32_selftest_kernel<<<dim3((n + 255) / 256), dim3(256), 0, st>>>(d, n, d + n,
                                                                  d + 2 * (size_t)n);
    HIP_TRY(hipStreamSynchronize(st));
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

int rt_debug_set_tile_variant(rt_ctx* ctx, int variant) {
    if (!ctx || variant < 0 || variant > 2) return RT_ERR_INVALID_ARG;
    ctx->tile_variant = variant;
    return RT_OK;
}

// The wide-tile (128x2) build's prep for the host-side culling tests.
int rt_debug_triangle_box_wide(const float v0[3], const float v1[3], const float v2[3],
                               const float dir[4], int32_t width, int32_t row_begin,
                               int32_t row_end, int32_t box_out[4], float cls_out[8]) {
    wide::TriRec r{};
    wide::Box b{};
    wide::Cls k{};
    bool bad = false;
    const bool ok = wide::prep_triangle(v0, v1, v2, dir[0], dir[1], dir[2], width, row_begin,
                                          row_end, &r, &b, &k, &bad);
    box_out[0] = b.x0; box_out[1] = b.y0; box_out[2] = b.x1; box_out[3] = b.y1;
    if (cls_out) std::memcpy(cls_out, &k, sizeof k);
    return ok ? 1 : 0;
}

int rt_debug_tile_shape_wide(int32_t* w, int32_t* h) {
    if (!w || !h) return RT_ERR_INVALID_ARG;
    *w = wide::kWaveTile;
    *h = wide::kWaveTileH;
    return RT_OK;
}

int rt_debug_set_coarse_cull(rt_ctx* ctx, int enable) {
    if (!ctx) return RT_ERR_INVALID_ARG;
    ctx->coarse_cull = enable < 0 ? RT_COARSE_CULL : enable;  // < 0: the default
    return RT_OK;
}

int rt_debug_set_coarse_cull_tri(rt_ctx* ctx, int min_candidates) {
    if (!ctx) return RT_ERR_INVALID_ARG;
    ctx->coarse_cull_tri = min_candidates < 0 ? RT_COARSE_CULL_TRI : min_candidates;
    ctx->coarse_cull_tri_rgba8 = min_candidates < 0 ? RT_COARSE_CULL_TRI_RGBA8 : min_candidates;
    return RT_OK;
}

int rt_debug_set_coarse_cull_overdraw(rt_ctx* ctx, int frames) {
    if (!ctx) return RT_ERR_INVALID_ARG;
    ctx->coarse_cull_overdraw = frames < 0 ? RT_COARSE_CULL_OVERDRAW : (unsigned)frames;
    ctx->coarse_cull_overdraw_rgba8 =
        frames < 0 ? RT_COARSE_CULL_OVERDRAW_RGBA8 : (unsigned)frames;
    // an explicit gate applies to every band size (the tests force the cull
    // on small frames this way)
    ctx->coarse_cull_tri_bins = frames < 0 ? RT_COARSE_CULL_TRI_BINS : 0;
    return RT_OK;
}

// tri_t_bounds of the 16x16 build's prep output (the TriDepth model), for
// the host tests: fp64 bounds of the trace's computed t over pixels
// [xa, xb] x [ya, yb].
int rt_debug_triangle_t_bounds(const float v0[3], const float v1[3], const float v2[3],
                               const float dir[4], int32_t width, int32_t row_begin,
                               int32_t row_end, int32_t xa, int32_t xb, int32_t ya, int32_t yb,
                               double out[2]) {
    TriRec r{};
    TriDepth d{0.0, 0.0, 0.0, INFINITY, 0.0, 0.0};
    Box b{};
    Cls k{};
    bool bad = false;
    if (!prep_triangle(v0, v1, v2, dir[0], dir[1], dir[2], width, row_begin, row_end, &r, &b, &k,
                       &bad, &d))
        return 0;
    return tri_t_bounds(d, xa, xb, ya, yb, &out[0], &out[1]) ? 1 : 0;
}

int rt_debug_set_small_fused(rt_ctx* ctx, int enable) {
    if (!ctx || enable < 0 || enable > 2) return RT_ERR_INVALID_ARG;
    ctx->small_fused = enable;
    return RT_OK;
}

int rt_debug_set_trace_split(rt_ctx* ctx, int waves) {
    if (!ctx || !(waves == 0 || waves == 1 || waves == 2 || waves == 4)) return RT_ERR_INVALID_ARG;
    ctx->trace_split = waves;
    return RT_OK;
}

int rt_debug_set_coarse_waves(rt_ctx* ctx, int waves) {
    if (!ctx || !(waves == 0 || waves == 1 || waves == 2 || waves == 4 || waves == 8))
        return RT_ERR_INVALID_ARG;
    ctx->coarse_waves = waves;
    return RT_OK;
}

int rt_debug_last_overdraw(rt_ctx* ctx, double* frames) {
    if (!ctx || !frames) return RT_ERR_INVALID_ARG;
    *frames = 0.0;
    if (ctx->od_launches == 0 || ctx->od_area == 0) return RT_OK;
    HIP_TRY(hipSetDevice(ctx->device));
    HIP_TRY(hipDeviceSynchronize());
    unsigned long long w[2];
    HIP_TRY(hipMemcpy(w, ctx->flag + 2, sizeof w, hipMemcpyDeviceToHost));
    *frames = (double)w[(ctx->od_launches - 1u) & 1u] / (double)ctx->od_area;
    return RT_OK;
}

int rt_debug_set_trace_bin(rt_ctx* ctx, int mode) {
    if (!ctx || mode < 0 || mode > 2) return RT_ERR_INVALID_ARG;
    ctx->trace_bin = mode;
    return RT_OK;
}

int rt_debug_set_verdict_copy(rt_ctx* ctx, int copy) {
    if (!ctx || copy < 0 || copy > 1) return RT_ERR_INVALID_ARG;
    if (!copy && !ctx->od_verdict_map) return RT_ERR_UNSUPPORTED;
    ctx->od_verdict_dev = copy ? nullptr : ctx->od_verdict_map;
    return RT_OK;
}

int rt_debug_set_small_path(rt_ctx* ctx, int enable) {
    if (!ctx) return RT_ERR_INVALID_ARG;
    ctx->small_path = enable != 0;
    return RT_OK;
}

#if RT_DIAG
// Diagnostics build only (rt_hip_diag.h): select a trace-kernel ablation.
int rt_debug_set_trace_mode(rt_ctx* ctx, int mode) {
    if (!ctx || mode < 0 || mode > 4) return RT_ERR_INVALID_ARG;
    ctx->trace_mode = mode;
    return RT_OK;
}
#endif

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
