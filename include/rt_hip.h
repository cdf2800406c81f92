/*
 * rt_hip.h -- C ABI of the MI355X-native per-pixel ray tracer (librt_hip.so).
 *
 * Drop-in boundary for RichardHancock/OpenCL-Ray-Tracer's GPU trace path.
 * Each entry point names the reference code it replaces (paths relative to
 * /root/reference/RayTrace).  Plain pointers and sizes only; no HIP, torch or
 * glm types cross this boundary.
 *
 * Scene layout is the reference's own flattened layout
 * (MainState.cpp:646-658, MainState.h:99-106):
 *   sphere_origins  float4[num_spheres]     (x, y, z, w)
 *   sphere_radius   float [num_spheres]
 *   sphere_colours  float4[num_spheres]     (r, g, b, a)
 *   cube_vertices   float4[36 * num_cubes]  12 world-space triangles per cube
 *   cube_colours    float4[num_cubes]
 * Output frame (MainState.cpp:952-955, rayTracer.cl:198-201):
 *   RT_FORMAT_I32X4: int32[rows][width][4], truncated (int) r, g, b, a
 *   RT_FORMAT_RGBA8: uint32[rows][width], (uint8)r | (uint8)g<<8 |
 *                    (uint8)b<<16 | 0xFF<<24  (the Texture packing,
 *                    MainState.cpp:984-994, :1023-1037)
 */
#ifndef RT_HIP_H
#define RT_HIP_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define RT_ABI_VERSION 1

/* Status codes: 0 = success, negative = failure.  Replaces the reference's
 * print-and-continue cl_int handling (MainState.cpp:1101-1179 getErrorString,
 * :672-674 etc.): the caller decides what to do. */
enum {
    RT_OK = 0,
    RT_ERR_INVALID_ARG = -1,
    RT_ERR_NO_DEVICE = -2,
    RT_ERR_HIP = -3,
    RT_ERR_OUT_OF_MEMORY = -4,
    RT_ERR_UNSUPPORTED = -5
};

enum { RT_FORMAT_I32X4 = 0, RT_FORMAT_RGBA8 = 1 };

/* Kernel path selection (rt_render*, `path` field of rt_timing). */
enum {
    RT_PATH_AUTO = 0,    /* binned when its preconditions hold, else generic */
    RT_PATH_BINNED = 1,  /* implicit origins (x,y,0,1), ray_dir = (0,0,D,w) */
    RT_PATH_GENERIC = 2  /* any origins / direction, brute force per pixel */
};

/* The kernel that did a render's per-pixel work (rt_last_kernel). */
enum {
    RT_KERNEL_NONE = 0,         /* no render yet */
    RT_KERNEL_TRACE = 1,        /* prep_kernel -> coarse3_kernel -> trace3_kernel */
    RT_KERNEL_TRACE_SMALL = 2,  /* prep_kernel -> trace_small_kernel (<= 512 primitives) */
    RT_KERNEL_FRAME_SMALL = 3,  /* frame_small_kernel, one launch (<= 128 primitives) */
    RT_KERNEL_GENERIC = 4,      /* generic_kernel: explicit origins / any direction */
    RT_KERNEL_TRACE_SPLIT = 5,  /* prep_kernel -> coarse3_kernel -> trace3_split_kernel
                                   (small frames: several waves per wave tile) */
    RT_KERNEL_TRACE_BIN = 6     /* prep_kernel -> trace_bin_kernel (tiles bin themselves) */
};

typedef struct rt_scene {
    const float* sphere_origins;
    const float* sphere_radius;
    const float* sphere_colours;
    int32_t num_spheres;
    const float* cube_vertices;
    const float* cube_colours;
    int32_t num_cubes;
    /* float4[num_lights].  Carried for ABI completeness; the reference has no
     * lighting model (its "shade" is a depth ramp, MainState.cpp:396-407), so
     * lights never change the output. */
    const float* lights;
    int32_t num_lights;
} rt_scene;

typedef struct rt_timing {
    double total_us;    /* host wall time of the whole call (the reference's
                           timer scope, MainState.cpp:662-894) */
    double upload_us;   /* HIP events from the stream point after the scene
                           was packed into page-locked staging on the host
                           (that packing, a few us of memcpy, is NOT in it;
                           it is in total_us) to the first render kernel's
                           start: the one H2D scene DMA, the explicit-origin
                           upload, the non-finite flag's reset when its
                           generation wraps, and the gaps before the first
                           kernel.  With explicit origins on the automatic
                           path it also covers their on-device grid check (a
                           small kernel, a 4-byte read-back and a stream sync
                           before the render, so the two are serialised) */
    double kernel_us;   /* first render kernel's start to the last one's end,
                           the kernels' own dispatch-packet timestamps */
    double download_us; /* D2H frame copy, HIP events */
    int32_t path;       /* RT_PATH_BINNED or RT_PATH_GENERIC actually used */
} rt_timing;

typedef struct rt_ctx rt_ctx;

/* Replaces MainState::openCLInit (MainState.cpp:1181-1326): selects HIP
 * device `device_ordinal` and loads every kernel's code object onto it (the
 * counterpart of clBuildProgram / clCreateKernel, :1302-1320) and, once per
 * device and process, sets up the HIP runtime's staging for pageable
 * transfers, so the first render pays no loading.  The stream is created on first use and the
 * workspace grows on demand (or up front with rt_reserve).  One context per
 * device; not re-entrant per context. */
int rt_init(int device_ordinal, rt_ctx** out_ctx);

/* Sizes the context's workspace ahead of the first render of a frame of
 * `rows` x `width` pixels with this many spheres / cubes in `out_format`:
 * the host-API scene copy and frame, the binned path's records and
 * candidate lists, and the context's stream, on which it runs one small
 * pageable upload and download (the stream's first transfers).
 * Synchronous.  openCLInit does its one-time work before any trace
 * (MainState.cpp:1290-1320, outside the trace timer :662-894); after
 * rt_reserve the first rt_render of that size allocates nothing and pays no
 * setup.  Optional: rt_render reserves what it needs itself (before its
 * timed events).  Workspace only grows. */
int rt_reserve(rt_ctx* ctx, int32_t width, int32_t rows, int32_t num_spheres,
               int32_t num_cubes, int32_t out_format);

/* Releases everything rt_init / rt_render allocated (MainState.cpp:73-78). */
void rt_destroy(rt_ctx* ctx);

/* Replaces MainState::getErrorString (MainState.cpp:1101-1179). */
const char* rt_error_string(int status);

/* Replaces the body of MainState::executeRayTracerOpenCL
 * (MainState.cpp:641-934): buffer setup, the six scene/ray uploads, the
 * clEnqueueNDRangeKernel launch of rayTracer.cl::rayTracer and the blocking
 * map/readback.  Synchronous: on return `host_out` holds rows
 * [row_begin, row_end) of the width x height frame.
 *   ray_dir       float4, the reference passes (0,0,-1,-1) (MainState.cpp:37-39)
 *   ray_origins   NULL for the reference's implicit (x, y, 0, 1) grid
 *                 (MainState.cpp:44-50), else float4[width*height] (full
 *                 frame; only rows [row_begin, row_end) are uploaded, and
 *                 origins that are bit for bit that grid are recognised on
 *                 the device and keep the binned path)
 *   host_out      int32[4*width*rows] (I32X4) or uint32[width*rows] (RGBA8)
 *   timing        may be NULL
 * Empty scenes are legal (all pixels (0,0,0,255)). */
int rt_render(rt_ctx* ctx, const rt_scene* scene, const float ray_dir[4],
              const float* ray_origins, int32_t width, int32_t height,
              int32_t row_begin, int32_t row_end, int32_t out_format,
              void* host_out, rt_timing* timing);

/* Same as rt_render with an explicit path (RT_PATH_*).  RT_PATH_BINNED
 * returns RT_ERR_UNSUPPORTED when its preconditions do not hold. */
int rt_render_path(rt_ctx* ctx, const rt_scene* scene, const float ray_dir[4],
                   const float* ray_origins, int32_t width, int32_t height,
                   int32_t row_begin, int32_t row_end, int32_t out_format,
                   int32_t path, void* host_out, rt_timing* timing);

/* In-process multi-GPU render (SURVEY.md §8b/§8e rt_render_multi; the
 * reference is single-device, MainState.cpp:1241-1266).  Rows
 * [row_begin, row_end) are split into num_ctx contiguous bands of whole rows
 * (sizes differ by at most one row); band i is rendered on ctxs[i] (one
 * context per device, e.g. rt_init(i)) from its own host thread, straight
 * into its rows of host_out, so no gather step exists: the bands are
 * disjoint slices of the row-major frame (MainState.cpp:676 `pixels`).
 * Synchronous.  timings, if not NULL, gets one rt_timing per context
 * (zeroed for contexts left idle when num_ctx exceeds the row count).
 * Returns the first failing band's status. */
int rt_render_multi(rt_ctx* const* ctxs, int32_t num_ctx, const rt_scene* scene,
                    const float ray_dir[4], const float* ray_origins, int32_t width,
                    int32_t height, int32_t row_begin, int32_t row_end,
                    int32_t out_format, void* host_out, rt_timing* timings);

/* Device-resident variant (no reference counterpart; used by the multi-GPU
 * row-band driver and the benchmark): every pointer in `device_scene`,
 * `device_ray_origins` and `device_out` is a device pointer on the context's
 * device, `stream` is a hipStream_t (NULL = the context's stream).
 * Asynchronous: work is enqueued on `stream` and the call returns.
 * Renders on one context share its workspace (primitive records, candidate
 * lists): enqueue them on one stream, or synchronise before switching
 * streams.  Concurrent renders need one context each. */
int rt_render_device(rt_ctx* ctx, const rt_scene* device_scene,
                     const float ray_dir[4], const float* device_ray_origins,
                     int32_t width, int32_t height, int32_t row_begin,
                     int32_t row_end, int32_t out_format, int32_t path,
                     void* device_out, void* stream);

/* ---- multi-rank frame assembly over xGMI ------------- */
/* No reference counterpart (the reference is single-device,
 * MainState.cpp:1241-1266).  One process per GPU: the root allocates the
 * whole frame with rt_shared_alloc and hands the 64-byte handle to the
 * other ranks (any transport, e.g. a broadcast); each rank maps it with
 * rt_shared_open and passes `mapped + its first row` as rt_render_device's
 * device_out, so the trace kernel's framebuffer stores travel over xGMI
 * straight into the root's frame and no separate gather copy exists.
 * rt_shared_close unmaps an opened frame, rt_shared_free releases the
 * root's allocation (after every rank has closed it). */
typedef struct rt_ipc_handle {
    unsigned char bytes[64];
} rt_ipc_handle;
int rt_shared_alloc(rt_ctx* ctx, int64_t bytes, void** device_ptr, rt_ipc_handle* handle);
int rt_shared_open(rt_ctx* ctx, const rt_ipc_handle* handle, void** device_ptr);
int rt_shared_close(rt_ctx* ctx, void* device_ptr);
int rt_shared_free(rt_ctx* ctx, void* device_ptr);

/* Page-lock (and unlock) a caller-owned host buffer, e.g. the app's
 * `pixels` vector (MainState.cpp:215, :676), so that rt_render's frame
 * download is a direct DMA at the PCIe link rate instead of a staged copy.
 * Portable: every context / device may use it.  The reference maps and
 * copies an OpenCL buffer instead (MainState.cpp:876-907). */
int rt_host_register(void* host_ptr, int64_t bytes);
int rt_host_unregister(void* host_ptr);

/* Per-kernel HIP-event profiling of rt_render_device / rt_render launches.
 * rt_profile_enable(ctx, 1) starts recording; rt_profile_read synchronises,
 * returns the summed milliseconds of the prep, bin and trace kernels and the
 * number of renders recorded, then resets the accumulators. */
int rt_profile_enable(rt_ctx* ctx, int enable);
int rt_profile_read(rt_ctx* ctx, double* prep_ms, double* bin_ms,
                    double* trace_ms, int32_t* n_renders);

/* The kernel (RT_KERNEL_*) the last render enqueued on this context did
 * its per-pixel work with (for reports: which path actually ran). */
int rt_last_kernel(rt_ctx* ctx, int32_t* kernel);

/* Device facts for reporting (HBM bytes, CU count, name). */
int rt_device_info(rt_ctx* ctx, char* name, int32_t name_len, int32_t* n_cu,
                   int64_t* total_mem);

/* ---- host-side scene helpers (no GPU needed) ------------------------- */

/* Cube, Cube.cpp:6-83: unit cube, scale, rotate (Rz*Ry*Rx, radians),
 * translate, in place on float4[36]. */
void rt_cube_init(float vertices[144]);
void rt_cube_scale(float vertices[144], float sx, float sy, float sz);
void rt_cube_rotate(float vertices[144], float rx, float ry, float rz);
void rt_cube_translate(float vertices[144], float tx, float ty, float tz);
/* Utility::convertAngleToRadian, Utility.cpp:343-347 */
float rt_deg_to_rad(float degrees);
/* rayDir = perspective(45, 4/3, 0, 100) * (0,0,1,1), MainState.cpp:37-39 */
void rt_primary_ray_dir(float out[4]);

/* MainState::createScene1/2/3 (MainState.cpp:419-639) into caller arrays of
 * capacity 100 spheres / 100 cubes; Random::init(seed) = srand(seed). */
int rt_scene_reference(int32_t scene_id, uint32_t seed, float* sphere_origins,
                       float* sphere_radius, float* sphere_colours,
                       float* cube_vertices, float* cube_colours,
                       int32_t* num_spheres, int32_t* num_cubes);

/* Synthetic N-sphere / M-cube scene (SURVEY.md §8d distributions, seeded
 * splitmix64, object scale k: 1 = sparse, width/640 = dense). */
int rt_scene_synthetic(int32_t width, int32_t height, int32_t num_spheres,
                       int32_t num_cubes, uint64_t seed, float k,
                       float* sphere_origins, float* sphere_radius,
                       float* sphere_colours, float* cube_vertices,
                       float* cube_colours);

/* ---- scene build on the device ---------------- */

/* One Cube method call (Cube.cpp:53-83): scale(vec3), rotate(vec3) with
 * angles in RADIANS (Rz * Ry * Rx, as Cube::rotate), translate(vec3). */
enum { RT_CUBE_SCALE = 1, RT_CUBE_ROTATE = 2, RT_CUBE_TRANSLATE = 3 };
typedef struct rt_cube_op {
    int32_t op;
    float x, y, z;
} rt_cube_op;

/* Replaces building `cubes` on the host (Cube::Cube + its transform calls,
 * MainState.cpp:434-593, :617-638) followed by the vertex upload of
 * executeRayTracerOpenCL (MainState.cpp:646-658, :796-816).  Cube c starts
 * from device_vertices_in[36c .. 36c+35] (float4), or from Cube::Cube's unit
 * cube when device_vertices_in is NULL, and applies
 * device_ops[device_op_offsets[c] .. device_op_offsets[c+1]) in order; the
 * result goes to device_vertices_out (float4[36 * num_cubes], may equal
 * device_vertices_in).  Bit-identical to the rt_cube_* host functions (glibc
 * cosf/sinf restated on the device).  All pointers are device pointers;
 * asynchronous on `stream` (NULL = the context's stream). */
int rt_cube_build_device(rt_ctx* ctx, const rt_cube_op* device_ops,
                         const int32_t* device_op_offsets, int32_t num_cubes,
                         const float* device_vertices_in,
                         float* device_vertices_out, void* stream);

/* rt_scene_synthetic built on the device into device arrays: bit-identical
 * arrays, no host build or upload.  Asynchronous on `stream`. */
int rt_scene_synthetic_device(rt_ctx* ctx, int32_t width, int32_t height,
                              int32_t num_spheres, int32_t num_cubes,
                              uint64_t seed, float k, float* sphere_origins,
                              float* sphere_radius, float* sphere_colours,
                              float* cube_vertices, float* cube_colours,
                              void* stream);

/* Texture conversion (MainState.cpp:1023-1037) on the host. */
void rt_pack_rgba8(const int32_t* frame, int64_t n_pixels, uint32_t* out);

/* Known-answer checksum of a frame: FNV-1a-64 over its 32-bit words in
 * memory order (`h ^= w; h *= 0x100000001b3`), starting from `basis`
 * (RT_FNV1A64_BASIS; the survey's probe of the reference's CPU frames,
 * SURVEY.md §8c, started from 1469598103934665603).  No reference
 * counterpart: the app never checks its frame.  Used by the headless driver,
 * the benchmark's frame check against the committed fixtures and the tests. */
#define RT_FNV1A64_BASIS 0xcbf29ce484222325ull
uint64_t rt_fnv1a64(const void* words, int64_t n_words, uint64_t basis);

/* Library / ABI version. */
int rt_abi_version(void);

#ifdef __cplusplus
}
#endif
#endif /* RT_HIP_H */
