// rt_args.cpp -- host-only argument checks and pointer / size arithmetic of
// the C ABI (include/rt_args.h).  Plain C++, no HIP: the library links it,
// and the sanitizer build (Makefile `asan`) runs it under
// -fsanitize=address,undefined with the scene helpers and the oracle.
#include "rt_args.h"

namespace rt_args {

namespace {
size_t align_up(size_t v, size_t a) { return (v + a - 1) / a * a; }
}  // namespace

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

int check_reserve(int32_t width, int32_t rows, int32_t num_spheres, int32_t num_cubes,
                  int32_t fmt) {
    if (width <= 0 || rows <= 0 || width > (1 << 24) || rows > (1 << 24) || num_spheres < 0 ||
        num_cubes < 0 || (int64_t)12 * num_cubes + num_spheres > (int64_t)1 << 30 ||
        (fmt != RT_FORMAT_I32X4 && fmt != RT_FORMAT_RGBA8))
        return RT_ERR_INVALID_ARG;
    return RT_OK;
}

size_t frame_bytes(int32_t width, int32_t rows, int32_t fmt) {
    return (size_t)width * (size_t)rows * (fmt == RT_FORMAT_I32X4 ? 16u : 4u);
}

SceneLayout scene_layout(int32_t num_spheres, int32_t num_cubes) {
    const size_t ns = (size_t)num_spheres, nc = (size_t)num_cubes;
    SceneLayout l;
    l.sphere_origins = 0;
    l.sphere_radius = align_up(16 * ns, 256);
    l.sphere_colours = l.sphere_radius + align_up(4 * ns, 256);
    l.cube_vertices = l.sphere_colours + align_up(16 * ns, 256);
    l.cube_colours = l.cube_vertices + align_up(16 * 36 * nc, 256);
    l.bytes = l.cube_colours + align_up(16 * nc, 256) + 256;
    return l;
}

const float* band_origins(const float* origins, int32_t width, int32_t row_begin) {
    return origins ? origins + (size_t)4 * (size_t)width * (size_t)row_begin : nullptr;
}

}  // namespace rt_args
