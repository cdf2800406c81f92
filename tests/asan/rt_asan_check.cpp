// rt_asan_check.cpp -- host-side sanitizer run (SURVEY.md §5 "race detection
// / sanitizers"): built by `make -C opencl-ray-tracer_amd/csrc asan` with
// -fsanitize=address,undefined and run by tests/test_asan.py.
//
// Exercises, on exactly-sized heap arrays so that any overrun is reported:
//   - the scene helpers of the C ABI (csrc/rt_scene.cpp): rt_scene_reference
//     into its documented capacity of 100, rt_scene_synthetic, rt_cube_*,
//     rt_pack_rgba8 -- each against the oracle's own restatement;
//   - the host half of the ABI's argument checking and pointer arithmetic
//     (csrc/rt_args.cpp): check_args edge cases (empty scenes with NULL
//     arrays, the reference's unguarded &v[0] of MainState.cpp:765 / :814),
//     the device scene layout (MainState.cpp:666-743), the band offset into
//     a full-frame origin array (`ray_origins + 4*width*row_begin`);
//   - the oracle's whole-frame, row-band, threaded and row-sample paths
//     (oracle/rt_oracle.c) on small frames, including empty scenes.
// Exit 0 and "asan check ok" on success; a sanitizer report aborts.
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <vector>

#include "rt_args.h"
#include "rt_hip.h"
extern "C" {
#include "rt_oracle.h"
}

namespace {

int failures = 0;

#define CHECK(cond)                                                              \
    do {                                                                         \
        if (!(cond)) {                                                           \
            std::fprintf(stderr, "%s:%d: check failed: %s\n", __FILE__, __LINE__, \
                         #cond);                                                 \
            ++failures;                                                          \
        }                                                                        \
    } while (0)

// An exactly-sized heap array (no slack for an overrun to land in).
template <typename T>
struct Exact {
    std::unique_ptr<T[]> p;
    size_t n;
    explicit Exact(size_t count) : p(count ? new T[count]() : nullptr), n(count) {}
    T* get() { return p.get(); }
};

struct SceneArrays {
    Exact<float> so, sr, sc, cv, cc;
    int32_t ns = 0, nc = 0;
    SceneArrays(size_t cap_s, size_t cap_c)
        : so(4 * cap_s), sr(cap_s), sc(4 * cap_s), cv(144 * cap_c), cc(4 * cap_c) {}
    rt_scene view() {
        return rt_scene{so.get(), sr.get(), sc.get(), ns, cv.get(), cc.get(), nc, nullptr, 0};
    }
};

bool same_floats(const float* a, const float* b, size_t n) {
    return n == 0 || std::memcmp(a, b, n * sizeof(float)) == 0;
}

void reference_scenes() {
    for (int id = 1; id <= 3; ++id) {
        for (uint32_t seed : {1u, 7u}) {
            SceneArrays a(100, 100), b(100, 100);
            CHECK(rt_scene_reference(id, seed, a.so.get(), a.sr.get(), a.sc.get(), a.cv.get(),
                                     a.cc.get(), &a.ns, &a.nc) == RT_OK);
            CHECK(orc_scene_reference(id, seed, 1, b.so.get(), b.sr.get(), b.sc.get(), b.cv.get(),
                                      b.cc.get(), &b.ns, &b.nc) == 0);
            CHECK(a.ns == b.ns && a.nc == b.nc);
            CHECK(same_floats(a.so.get(), b.so.get(), 4 * (size_t)a.ns));
            CHECK(same_floats(a.sr.get(), b.sr.get(), (size_t)a.ns));
            CHECK(same_floats(a.cv.get(), b.cv.get(), 144 * (size_t)a.nc));
            CHECK(same_floats(a.cc.get(), b.cc.get(), 4 * (size_t)a.nc));
        }
    }
    SceneArrays a(100, 100);
    CHECK(rt_scene_reference(0, 1, a.so.get(), a.sr.get(), a.sc.get(), a.cv.get(), a.cc.get(),
                             &a.ns, &a.nc) == RT_ERR_INVALID_ARG);
    CHECK(rt_scene_reference(4, 1, a.so.get(), a.sr.get(), a.sc.get(), a.cv.get(), a.cc.get(),
                             &a.ns, &a.nc) == RT_ERR_INVALID_ARG);
}

void synthetic_scenes() {
    struct Case { int32_t w, h, ns, nc; uint64_t seed; float k; };
    const Case cases[] = {{512, 512, 4, 1, 1, 0.8f}, {1, 1, 0, 0, 2, 1.0f}, {7, 3, 0, 5, 3, 1.0f},
                          {64, 64, 33, 0, 4, 0.1f},  {1920, 1080, 16, 4, 2, 3.0f}};
    for (const Case& c : cases) {
        SceneArrays a((size_t)c.ns, (size_t)c.nc), b((size_t)c.ns, (size_t)c.nc);
        CHECK(rt_scene_synthetic(c.w, c.h, c.ns, c.nc, c.seed, c.k, a.so.get(), a.sr.get(),
                                 a.sc.get(), a.cv.get(), a.cc.get()) == RT_OK);
        orc_scene_synthetic(c.w, c.h, c.ns, c.nc, c.seed, c.k, b.so.get(), b.sr.get(), b.sc.get(),
                            b.cv.get(), b.cc.get());
        CHECK(same_floats(a.so.get(), b.so.get(), 4 * (size_t)c.ns));
        CHECK(same_floats(a.sr.get(), b.sr.get(), (size_t)c.ns));
        CHECK(same_floats(a.sc.get(), b.sc.get(), 4 * (size_t)c.ns));
        CHECK(same_floats(a.cv.get(), b.cv.get(), 144 * (size_t)c.nc));
        CHECK(same_floats(a.cc.get(), b.cc.get(), 4 * (size_t)c.nc));
    }
    CHECK(rt_scene_synthetic(0, 10, 1, 1, 1, 1.0f, nullptr, nullptr, nullptr, nullptr, nullptr) ==
          RT_ERR_INVALID_ARG);
}

void cubes() {
    Exact<float> a(144), b(144);
    rt_cube_init(a.get());
    orc_cube_init(b.get());
    rt_cube_scale(a.get(), 5, 6, 7);
    orc_cube_scale(b.get(), 5, 6, 7);
    rt_cube_rotate(a.get(), 0.3f, -1.1f, 2.0f);
    orc_cube_rotate(b.get(), 0.3f, -1.1f, 2.0f);
    rt_cube_translate(a.get(), 100, 50, -60);
    orc_cube_translate(b.get(), 100, 50, -60);
    CHECK(same_floats(a.get(), b.get(), 144));
}

void pack() {
    for (int64_t n : {0, 1, 3, 257}) {
        Exact<int32_t> frame((size_t)(4 * n));
        for (int64_t i = 0; i < 4 * n; ++i) frame.get()[i] = (int32_t)(i * 37 % 700) - 200;
        Exact<uint32_t> a((size_t)n), b((size_t)n);
        rt_pack_rgba8(frame.get(), n, a.get());
        orc_pack_rgba8(frame.get(), n, b.get());
        CHECK(n == 0 || std::memcmp(a.get(), b.get(), (size_t)n * 4) == 0);
    }
}

void args() {
    using rt_args::check_args;
    rt_scene empty{nullptr, nullptr, nullptr, 0, nullptr, nullptr, 0, nullptr, 0};
    // zero spheres / cubes with NULL arrays are legal
    CHECK(check_args(&empty, 640, 480, 0, 480, RT_FORMAT_I32X4) == RT_OK);
    CHECK(check_args(&empty, 1, 1, 0, 1, RT_FORMAT_RGBA8) == RT_OK);
    CHECK(check_args(nullptr, 640, 480, 0, 480, RT_FORMAT_I32X4) == RT_ERR_INVALID_ARG);
    // a positive count with a NULL array
    rt_scene s = empty;
    s.num_spheres = 1;
    CHECK(check_args(&s, 8, 8, 0, 8, 0) == RT_ERR_INVALID_ARG);
    s = empty;
    s.num_cubes = 1;
    CHECK(check_args(&s, 8, 8, 0, 8, 0) == RT_ERR_INVALID_ARG);
    s = empty;
    s.num_lights = -1;
    CHECK(check_args(&s, 8, 8, 0, 8, 0) == RT_ERR_INVALID_ARG);
    // rows, sizes, format
    CHECK(check_args(&empty, 8, 8, 8, 8, 0) == RT_ERR_INVALID_ARG);   // empty range
    CHECK(check_args(&empty, 8, 8, -1, 8, 0) == RT_ERR_INVALID_ARG);
    CHECK(check_args(&empty, 8, 8, 0, 9, 0) == RT_ERR_INVALID_ARG);
    CHECK(check_args(&empty, 0, 8, 0, 8, 0) == RT_ERR_INVALID_ARG);
    CHECK(check_args(&empty, (1 << 24) + 1, 1, 0, 1, 0) == RT_ERR_INVALID_ARG);
    CHECK(check_args(&empty, 1 << 24, 1, 0, 1, 0) == RT_OK);
    CHECK(check_args(&empty, 8, 8, 0, 8, 2) == RT_ERR_INVALID_ARG);
    // 12 M + N beyond 2^30 (the count, not the arrays, is checked)
    float dummy[4] = {0, 0, 0, 0};
    s = empty;
    s.cube_vertices = s.cube_colours = dummy;
    s.num_cubes = (1 << 30) / 12 + 1;
    CHECK(check_args(&s, 8, 8, 0, 8, 0) == RT_ERR_INVALID_ARG);
    s.num_cubes = INT32_MAX;
    CHECK(check_args(&s, 8, 8, 0, 8, 0) == RT_ERR_INVALID_ARG);
    CHECK(rt_args::check_reserve(640, 480, 0, 0, RT_FORMAT_I32X4) == RT_OK);
    CHECK(rt_args::check_reserve(640, 0, 0, 0, RT_FORMAT_I32X4) == RT_ERR_INVALID_ARG);
    CHECK(rt_args::check_reserve(640, 480, -1, 0, RT_FORMAT_I32X4) == RT_ERR_INVALID_ARG);
    CHECK(rt_args::check_reserve(640, 480, 0, INT32_MAX, RT_FORMAT_I32X4) == RT_ERR_INVALID_ARG);
    CHECK(rt_args::frame_bytes(1 << 14, 1 << 14, RT_FORMAT_I32X4) == (size_t)1 << 32);
    CHECK(rt_args::frame_bytes(3, 2, RT_FORMAT_RGBA8) == 24);
}

// The device scene copy, simulated on the host: every array copied to its
// layout offset inside a buffer of exactly layout.bytes.
void layout() {
    const int32_t counts[][2] = {{0, 0}, {1, 0}, {0, 1}, {3, 7}, {100, 100}, {4096, 0}};
    for (const auto& c : counts) {
        const rt_args::SceneLayout l = rt_args::scene_layout(c[0], c[1]);
        const size_t ns = (size_t)c[0], nc = (size_t)c[1];
        CHECK(l.sphere_origins % 256 == 0 && l.sphere_radius % 256 == 0 &&
              l.sphere_colours % 256 == 0 && l.cube_vertices % 256 == 0 &&
              l.cube_colours % 256 == 0);
        CHECK(l.sphere_radius >= l.sphere_origins + 16 * ns);
        CHECK(l.sphere_colours >= l.sphere_radius + 4 * ns);
        CHECK(l.cube_vertices >= l.sphere_colours + 16 * ns);
        CHECK(l.cube_colours >= l.cube_vertices + 576 * nc);
        CHECK(l.bytes >= l.cube_colours + 16 * nc);
        SceneArrays a(ns, nc);
        Exact<char> dev(l.bytes);
        if (ns) {
            std::memcpy(dev.get() + l.sphere_origins, a.so.get(), 16 * ns);
            std::memcpy(dev.get() + l.sphere_radius, a.sr.get(), 4 * ns);
            std::memcpy(dev.get() + l.sphere_colours, a.sc.get(), 16 * ns);
        }
        if (nc) {
            std::memcpy(dev.get() + l.cube_vertices, a.cv.get(), 576 * nc);
            std::memcpy(dev.get() + l.cube_colours, a.cc.get(), 16 * nc);
        }
    }
}

// rt_render's band upload of explicit origins: rows [rb, re) of a full-frame
// float4 array, read through rt_args::band_origins.
void band_origins() {
    const int32_t w = 37, h = 23;
    Exact<float> org((size_t)4 * w * h);
    for (int32_t y = 0; y < h; ++y)
        for (int32_t x = 0; x < w; ++x) {
            float* o = org.get() + 4 * ((size_t)y * w + x);
            o[0] = (float)x; o[1] = (float)y; o[2] = 0.0f; o[3] = 1.0f;
        }
    CHECK(rt_args::band_origins(nullptr, w, 5) == nullptr);
    const int32_t bands[][2] = {{0, h}, {0, 1}, {h - 1, h}, {5, 17}, {17, h}};
    for (const auto& b : bands) {
        const float* p = rt_args::band_origins(org.get(), w, b[0]);
        const size_t n = (size_t)4 * w * (b[1] - b[0]);
        Exact<float> copy(n);
        std::memcpy(copy.get(), p, n * sizeof(float));  // the upload's read
        CHECK(copy.get()[0] == 0.0f && copy.get()[1] == (float)b[0]);
        CHECK(copy.get()[n - 4] == (float)(w - 1) && copy.get()[n - 3] == (float)(b[1] - 1));
    }
}

void oracle_paths() {
    const int32_t w = 48, h = 36;
    float dir[4];
    orc_ray_dir(dir);
    SceneArrays a(100, 100);
    CHECK(orc_scene_reference(1, 1, 1, a.so.get(), a.sr.get(), a.sc.get(), a.cv.get(), a.cc.get(),
                              &a.ns, &a.nc) == 0);
    // scale scene 1 (640x480 units) into the small frame: the reference's
    // arrays, only fewer pixels
    Exact<int32_t> whole((size_t)4 * w * h);
    orc_trace(w, h, 0, h, dir, nullptr, a.ns, a.so.get(), a.sr.get(), a.sc.get(), a.nc, a.cv.get(),
              a.cc.get(), whole.get());
    // row bands equal the whole frame's rows
    const int32_t bands[][2] = {{0, 1}, {3, 20}, {h - 1, h}};
    for (const auto& b : bands) {
        Exact<int32_t> band((size_t)4 * w * (b[1] - b[0]));
        orc_trace(w, h, b[0], b[1], dir, nullptr, a.ns, a.so.get(), a.sr.get(), a.sc.get(), a.nc,
                  a.cv.get(), a.cc.get(), band.get());
        CHECK(std::memcmp(band.get(), whole.get() + (size_t)4 * w * b[0], band.n * 4) == 0);
    }
    // threaded, more threads than rows of a band
    Exact<int32_t> mt((size_t)4 * w * h);
    orc_trace_mt(w, h, 0, h, dir, nullptr, a.ns, a.so.get(), a.sr.get(), a.sc.get(), a.nc,
                 a.cv.get(), a.cc.get(), mt.get(), 5);
    CHECK(std::memcmp(mt.get(), whole.get(), mt.n * 4) == 0);
    Exact<int32_t> mt2((size_t)4 * w * 2);
    orc_trace_mt(w, h, 10, 12, dir, nullptr, a.ns, a.so.get(), a.sr.get(), a.sc.get(), a.nc,
                 a.cv.get(), a.cc.get(), mt2.get(), 7);
    CHECK(std::memcmp(mt2.get(), whole.get() + (size_t)4 * w * 10, mt2.n * 4) == 0);
    // the CPU baseline's row sample
    const int32_t rows[] = {35, 0, 17};
    Exact<int32_t> rs((size_t)4 * w * 3);
    orc_trace_rows_mt(w, h, rows, 3, dir, nullptr, a.ns, a.so.get(), a.sr.get(), a.sc.get(), a.nc,
                      a.cv.get(), a.cc.get(), rs.get(), 2);
    for (int i = 0; i < 3; ++i)
        CHECK(std::memcmp(rs.get() + (size_t)4 * w * i, whole.get() + (size_t)4 * w * rows[i],
                          (size_t)16 * w) == 0);
    // explicit full-frame origins equal to the implicit grid, and a band
    Exact<float> org((size_t)4 * w * h);
    for (int32_t y = 0; y < h; ++y)
        for (int32_t x = 0; x < w; ++x) {
            float* o = org.get() + 4 * ((size_t)y * w + x);
            o[0] = (float)x; o[1] = (float)y; o[2] = 0.0f; o[3] = 1.0f;
        }
    Exact<int32_t> eo((size_t)4 * w * (h - 30));
    orc_trace(w, h, 30, h, dir, org.get(), a.ns, a.so.get(), a.sr.get(), a.sc.get(), a.nc,
              a.cv.get(), a.cc.get(), eo.get());
    CHECK(std::memcmp(eo.get(), whole.get() + (size_t)4 * w * 30, eo.n * 4) == 0);
    // empty scenes with NULL arrays: every pixel (0, 0, 0, 255)
    Exact<int32_t> e((size_t)4 * w * h);
    orc_trace(w, h, 0, h, dir, nullptr, 0, nullptr, nullptr, nullptr, 0, nullptr, nullptr, e.get());
    bool black = true;
    for (size_t i = 0; i < e.n; ++i) black &= e.get()[i] == ((i % 4 == 3) ? 255 : 0);
    CHECK(black);
    // spheres only / cubes only with the other array NULL
    Exact<int32_t> so((size_t)4 * w * h), co((size_t)4 * w * h);
    orc_trace(w, h, 0, h, dir, nullptr, a.ns, a.so.get(), a.sr.get(), a.sc.get(), 0, nullptr,
              nullptr, so.get());
    orc_trace(w, h, 0, h, dir, nullptr, 0, nullptr, nullptr, nullptr, a.nc, a.cv.get(), a.cc.get(),
              co.get());
    // the reference's known-answer statistics need 640x480; here only the FNV
    // of the small frame is printed for the log
    std::printf("oracle 48x36 scene-1 fnv %016llx\n",
                (unsigned long long)orc_fnv1a_i32(whole.get(), (int64_t)whole.n));
}

}  // namespace

int main(int argc, char** argv) {
    if (argc > 1 && std::strcmp(argv[1], "--control-overrun") == 0) {
        // negative control (tests/test_asan.py): the sanitizer must report
        // this one-element overrun of an exactly-sized array
        Exact<float> a(4);
        volatile float* p = a.get();
        std::printf("%f\n", (double)p[4 + (argc > 2 ? 1 : 0)]);
        return 0;
    }
    reference_scenes();
    synthetic_scenes();
    cubes();
    pack();
    args();
    layout();
    band_origins();
    oracle_paths();
    if (failures) {
        std::fprintf(stderr, "%d checks failed\n", failures);
        return 1;
    }
    std::printf("asan check ok\n");
    return 0;
}
