/*
 * rt_oracle.h -- TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement of the reference's serial ray tracer
 * (RichardHancock/OpenCL-Ray-Tracer, RayTrace/states/MainState.cpp:257-408,
 * :936-972) plus its scene construction (MainState.cpp:419-639, Cube.cpp:6-83,
 * glm 0.9.6.1 gtc/matrix_transform.inl, detail/type_mat4x4.inl,
 * detail/func_geometric.inl, misc/Random.cpp:29-42, misc/Utility.cpp:109-116,
 * :343-347).
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may
 * load this library, and only as the checker / CPU baseline.  The product
 * path (librt_hip.so) never links or calls it.
 *
 * Parity pinning: see the header of rt_oracle.c.
 */
#ifndef RT_ORACLE_H
#define RT_ORACLE_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- Cube packing: 36 float4 vertices (12 triangles), Cube.cpp:6-46 ---- */
void orc_cube_init(float verts[144]);
void orc_cube_scale(float verts[144], float sx, float sy, float sz);      /* Cube.cpp:65-73 */
void orc_cube_rotate(float verts[144], float rx, float ry, float rz);     /* Cube.cpp:53-63 */
void orc_cube_translate(float verts[144], float tx, float ty, float tz);  /* Cube.cpp:75-83 */
float orc_deg2rad(float deg);                                             /* Utility.cpp:343-347 */

/* Random::init / Random::getFloat (Random.cpp:10-42) on glibc rand(). */
void orc_srand(unsigned seed);
float orc_get_float(float mn, float mx);

/* ---- the primary ray direction, MainState.cpp:37-39 ---- */
void orc_ray_dir(float out[4]);

/* ---- scenes ----
 * Reference scenes 1..3 (MainState.cpp:419-639).  Scenes 2 and 3 draw from
 * glibc rand() after srand(seed) (Random.cpp:10-17).  `rtl` selects the
 * evaluation order of the unspecified-order Random::getFloat() arguments
 * inside one glm::vec4/vec3 constructor call: 1 = right-to-left (what g++
 * on x86-64 does), 0 = left-to-right.
 * Capacity: spheres <= 100, cubes <= 100.  Returns 0 on success. */
int orc_scene_reference(int scene_id, unsigned seed, int rtl,
                        float* sphere_origins, float* sphere_radius,
                        float* sphere_colours, float* cube_vertices,
                        float* cube_colours, int32_t* n_spheres,
                        int32_t* n_cubes);

/* Synthetic N-sphere / M-cube scene: splitmix64 stream,
 * k = object scale factor (1 = sparse reference units, W/640 = dense). */
void orc_scene_synthetic(int32_t width, int32_t height, int32_t n_spheres,
                         int32_t n_cubes, uint64_t seed, float k,
                         float* sphere_origins, float* sphere_radius,
                         float* sphere_colours, float* cube_vertices,
                         float* cube_colours);

/* ---- per-ray primitives ---- */
int orc_intersect_tri(const double orig[3], const double dir[3],
                      const double v0[3], const double v1[3],
                      const double v2[3], double* t, double* u, double* v);
float orc_intersect_sphere(const float o[4], const float d[4], float radius,
                           const float c[4]);

/* ---- one pixel / a band of rows ----
 * Output is int32 RGBA per pixel, rows [row_begin,row_end) of a W-wide
 * frame, row-major.  ray_origins may be NULL (implicit (x,y,0,1),
 * MainState.cpp:44-50) or a full-frame float4[W*H] array. */
void orc_collide(const float origin[4], const float dir[4], int32_t n_spheres,
                 const float* sphere_origins, const float* sphere_radius,
                 const float* sphere_colours, int32_t n_cubes,
                 const float* cube_vertices, const float* cube_colours,
                 int32_t out[4]);
void orc_trace(int32_t width, int32_t height, int32_t row_begin,
               int32_t row_end, const float ray_dir[4],
               const float* ray_origins, int32_t n_spheres,
               const float* sphere_origins, const float* sphere_radius,
               const float* sphere_colours, int32_t n_cubes,
               const float* cube_vertices, const float* cube_colours,
               int32_t* out);
/* Same, over `n_threads` POSIX threads (row-interleaved), for the CPU baseline. */
void orc_trace_mt(int32_t width, int32_t height, int32_t row_begin,
                  int32_t row_end, const float ray_dir[4],
                  const float* ray_origins, int32_t n_spheres,
                  const float* sphere_origins, const float* sphere_radius,
                  const float* sphere_colours, int32_t n_cubes,
                  const float* cube_vertices, const float* cube_colours,
                  int32_t* out, int32_t n_threads);

/* The listed rows (any order), each into out[i] (n_rows x W x 4), over
 * `n_threads` threads: the CPU-baseline row sample. */
void orc_trace_rows_mt(int32_t width, int32_t height, const int32_t* rows,
                       int32_t n_rows, const float ray_dir[4],
                       const float* ray_origins, int32_t n_spheres,
                       const float* sphere_origins, const float* sphere_radius,
                       const float* sphere_colours, int32_t n_cubes,
                       const float* cube_vertices, const float* cube_colours,
                       int32_t* out, int32_t n_threads);

/* The reference's fp32 OpenCL kernel semantics (rayTracer.cl:37-202), the
 * same collide text as orc_trace in the kernel's arithmetic -- not the
 * parity target.  cl32: glm dot and x86 (int) (the survey probe's host
 * build, for the SURVEY.md F5 divergence pin); cl_gfx950: the kernel as
 * compiled for gfx950 by oracle/Makefile (device-library fma dot,
 * v_cvt_i32_f32), pinned against that kernel run on the GPU. */
void orc_trace_cl32(int32_t width, int32_t height, const float ray_dir[4],
                    int32_t n_spheres, const float* sphere_origins,
                    const float* sphere_radius, const float* sphere_colours,
                    int32_t n_cubes, const float* cube_vertices,
                    const float* cube_colours, int32_t* out);
void orc_trace_cl_gfx950(int32_t width, int32_t height, const float ray_dir[4],
                         const float* ray_origins, int32_t n_spheres,
                         const float* sphere_origins, const float* sphere_radius,
                         const float* sphere_colours, int32_t n_cubes,
                         const float* cube_vertices, const float* cube_colours,
                         int32_t* out);

/* Per-pixel hit masks of one triangle (orc_intersect_tri == 1) / one sphere
 * (passes the tca and distance tests) over [x0,x0+w) x [y0,y0+h). */
void orc_tri_grid(const float v0[3], const float v1[3], const float v2[3],
                  const float dir[4], int32_t x0, int32_t y0, int32_t w, int32_t h,
                  uint8_t* hits);
void orc_tri_t_grid(const float v0[3], const float v1[3], const float v2[3], const float dir[4],
                    int32_t x0, int32_t y0, int32_t w, int32_t h, double* ts);
void orc_sphere_grid(const float centre[4], float radius, const float dir[4],
                     int32_t x0, int32_t y0, int32_t w, int32_t h, uint8_t* hits);

/* FNV-1a-64 over the int32 stream (SURVEY.md §8c known-answer format). */
/* The host libm's sinf / cosf on n floats: what glm::rotate's std::cos /
 * std::sin (matrix_transform.inl:52-58) compute in the reference's CPU
 * build; the checker of the device's glibc restatement. */
void orc_libm_sincosf(const float* x, int64_t n, float* s, float* c);
uint64_t orc_fnv1a_i32(const int32_t* v, int64_t n);

/* Texture packing, MainState.cpp:1023-1037 + masks :984-994:
 * (uint8)r | (uint8)g<<8 | (uint8)b<<16 | 0xFF<<24 (SDL_MapRGB => opaque). */
void orc_pack_rgba8(const int32_t* frame, int64_t n_pixels, uint32_t* out);

#ifdef __cplusplus
}
#endif
#endif
