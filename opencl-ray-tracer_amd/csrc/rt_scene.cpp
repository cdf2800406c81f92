// rt_scene.cpp -- host-side scene construction for librt_hip.so.
//
// The reference builds its scenes on the host in float through glm 0.9.6.1
// (Cube.cpp:6-83, MainState.cpp:419-639) and hands the kernel world-space
// triangle vertices.  This file provides the same packing so a caller of the
// C ABI (and the headless driver / benchmark) can build the reference's
// scenes and the synthetic benchmark scenes without glm.  Compiled with
// -ffp-contract=off: each float operation is rounded once, in glm's order.
#include <cmath>
#include <cstdint>
#include <cstdlib>
#include <cstring>

#include "rt_hip.h"

namespace {

// Column-major 4x4, col[c][r], as glm::tmat4x4.
struct Mat4 {
    float col[4][4];
    static Mat4 identity() {
        Mat4 m{};
        for (int i = 0; i < 4; ++i) m.col[i][i] = 1.0f;
        return m;
    }
    // glm type_mat4x4.inl:596-607 -- (m0*v0 + m1*v1) + (m2*v2 + m3*v3)
    void apply(float* v) const {
        float r[4];
        for (int i = 0; i < 4; ++i) {
            const float lo = col[0][i] * v[0] + col[1][i] * v[1];
            const float hi = col[2][i] * v[2] + col[3][i] * v[3];
            r[i] = lo + hi;
        }
        std::memcpy(v, r, sizeof r);
    }
};

// glm matrix_transform.inl:52-85, with normalize() = v * (1/sqrt(dot(v,v))).
Mat4 rotate(const Mat4& m, float angle, const float axis_in[3]) {
    const float c = std::cos(angle);
    const float s = std::sin(angle);
    const float len2 = axis_in[0] * axis_in[0] + axis_in[1] * axis_in[1] + axis_in[2] * axis_in[2];
    const float inv_len = 1.0f / std::sqrt(len2);
    const float a[3] = {axis_in[0] * inv_len, axis_in[1] * inv_len, axis_in[2] * inv_len};
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
            out.col[j][r] = m.col[0][r] * rot[j][0] + m.col[1][r] * rot[j][1] + m.col[2][r] * rot[j][2];
    for (int r = 0; r < 4; ++r) out.col[3][r] = m.col[3][r];
    return out;
}

void transform_all(float* verts, const Mat4& m) {
    for (int i = 0; i < 36; ++i) m.apply(verts + 4 * i);
}

// Cube.cpp:10-45, the 36 corners of the unit cube's 12 triangles, encoded
// as 3-bit corner ids (bit0 = x, bit1 = y, bit2 = z; set bit = +1).
const unsigned char kCorners[36] = {
    0, 4, 6, 3, 0, 2, 5, 0, 1, 3, 1, 0, 0, 6, 2, 5, 4, 0,
    6, 4, 5, 7, 1, 3, 1, 7, 5, 7, 3, 2, 7, 2, 6, 7, 6, 5};

// Random::getFloat (Random.cpp:29-42) on glibc rand().
float glibc_uniform(float lo, float hi) {
    const float unit = static_cast<float>(std::rand()) / static_cast<float>(RAND_MAX);
    const float span = hi - lo;
    return lo + unit * span;
}

// The reference draws three getFloat() calls as arguments of one glm
// constructor; g++ on x86-64 evaluates those right to left.
void glibc_uniform3(const float lo[3], const float hi[3], float out[3]) {
    out[2] = glibc_uniform(lo[2], hi[2]);
    out[1] = glibc_uniform(lo[1], hi[1]);
    out[0] = glibc_uniform(lo[0], hi[0]);
}

const float kColLo[3] = {0.05f, 0.05f, 0.05f}, kColHi[3] = {1.0f, 1.0f, 1.0f};

struct Sink {
    float *so, *sr, *sc, *cv, *cc;
    int32_t ns = 0, nc = 0;
    void sphere(const float o[3], float r, const float col[3]) {
        float* p = so + 4 * ns;
        p[0] = o[0]; p[1] = o[1]; p[2] = o[2]; p[3] = 1.0f;
        sr[ns] = r;
        float* c = sc + 4 * ns;
        c[0] = col[0]; c[1] = col[1]; c[2] = col[2]; c[3] = 255.0f;
        ++ns;
    }
    float* cube(const float col[3]) {
        float* v = cv + 144 * nc;
        rt_cube_init(v);
        float* c = cc + 4 * nc;
        c[0] = col[0]; c[1] = col[1]; c[2] = col[2]; c[3] = 255.0f;
        ++nc;
        return v;
    }
};

// One scripted transform step of a hand-placed cube (MainState.cpp:434-593).
struct Step {
    char op;  // 's' scale, 'r' rotate (x,y,z in DEGREES unless raw), 't' translate
    float x, y, z;
    bool raw_z = false;  // cube9's rotate(vec3(rad(150), 0, 9.9f)) at :579
};

void run_steps(float* v, const Step* steps, int n) {
    for (int i = 0; i < n; ++i) {
        const Step& s = steps[i];
        if (s.op == 's') {
            rt_cube_scale(v, s.x, s.y, s.z);
        } else if (s.op == 't') {
            rt_cube_translate(v, s.x, s.y, s.z);
        } else {
            const float rx = s.x != 0.0f ? rt_deg_to_rad(s.x) : 0.0f;
            const float ry = s.y != 0.0f ? rt_deg_to_rad(s.y) : 0.0f;
            const float rz = s.raw_z ? s.z : (s.z != 0.0f ? rt_deg_to_rad(s.z) : 0.0f);
            rt_cube_rotate(v, rx, ry, rz);
        }
    }
}

struct FixedCube {
    float colour[3];
    Step steps[4];
};

// Cubes 1-4, identical in scenes 1 and 2 (MainState.cpp:434-461, :499-526).
const FixedCube kFixedCubes[4] = {
    {{1, 1, 0}, {{'s', 40, 40, 40}, {'r', 0, 0, 30}, {'r', 0, 30, 0}, {'t', 70, 60, -60}}},
    {{0, 1, 1}, {{'s', 30, 30, 30}, {'r', 0, 0, 80}, {'r', 0, 250, 0}, {'t', 150, 60, -70}}},
    {{0, 0, 1}, {{'s', 10, 10, 10}, {'r', 0, 0, 160}, {'r', 210, 0, 0}, {'t', 150, 400, -40}}},
    {{1, 0, 0}, {{'s', 50, 50, 50}, {'r', 0, 0, 80}, {'r', 0, 250, 0}, {'t', 450, 200, -80}}},
};

void build_scene1(Sink& k) {
    const float o0[3] = {300, 250, -85}, c0[3] = {0, 1, 1};
    const float o1[3] = {500, 250, -85}, c1[3] = {1, 0, 1};
    k.sphere(o0, 50.0f, c0);
    k.sphere(o1, 30.0f, c1);
    for (const FixedCube& fc : kFixedCubes) run_steps(k.cube(fc.colour), fc.steps, 4);
}

void build_scene2(Sink& k) {
    static const float o[8][3] = {{100, 150, -85}, {300, 400, -65}, {350, 150, -85},
                                  {200, 250, -85}, {200, 350, -45}, {600, 450, -125},
                                  {20, 450, -64},  {620, 250, -115}};
    static const float r[8] = {50, 30, 15, 25, 20, 42, 42, 32};
    for (int i = 0; i < 8; ++i) {
        float col[3];
        glibc_uniform3(kColLo, kColHi, col);
        k.sphere(o[i], r[i], col);
    }
    for (const FixedCube& fc : kFixedCubes) run_steps(k.cube(fc.colour), fc.steps, 4);
    // cubes 5-10, random colours (MainState.cpp:528-593)
    static const Step s5[] = {{'s', 30, 30, 30}, {'r', 170, 0, 0}, {'r', 0, 150, 0}, {'t', 450, 400, -60}};
    static const Step s6[] = {{'s', 50, 50, 50}, {'r', 0, 0, 80}, {'r', 350, 0, 0}, {'t', 50, 300, -100}};
    static const Step s7[] = {{'s', 70, 70, 70}, {'r', 160, 0, 0}, {'r', 0, 250, 0}, {'t', 530, 300, -100}};
    static const Step s8[] = {{'s', 25, 25, 25}, {'r', 0, 0, 190}, {'r', 0, 140, 0}, {'t', 230, 150, -40}};
    static const Step s9[] = {{'s', 50, 50, 50}, {'r', 0, 130, 0}, {'r', 150, 0, 9.9f, true},
                              {'r', 0, 0, 50}, {'t', 510, 50, -90}};
    static const Step s10[] = {{'s', 24, 24, 24}, {'r', 0, 0, 280}, {'r', 0, 20, 0}, {'t', 350, 340, -40}};
    const Step* scripts[6] = {s5, s6, s7, s8, s9, s10};
    const int lengths[6] = {4, 4, 4, 4, 5, 4};
    for (int i = 0; i < 6; ++i) {
        float col[3];
        glibc_uniform3(kColLo, kColHi, col);
        run_steps(k.cube(col), scripts[i], lengths[i]);
    }
}

void build_scene3(Sink& k) {
    static const float kPosLo[3] = {0.0f, 0.0f, 20.0f}, kPosHi[3] = {630.0f, 470.0f, 100.0f};
    static const float kCubeLo[3] = {0.0f, 0.0f, 30.0f}, kCubeHi[3] = {630.0f, 470.0f, 100.0f};
    for (int i = 0; i < 100; ++i) {  // MainState.cpp:599-615
        float p[3], col[3];
        glibc_uniform3(kPosLo, kPosHi, p);
        p[2] = -p[2];
        const float r = glibc_uniform(5.0f, 30.0f);
        glibc_uniform3(kColLo, kColHi, col);
        k.sphere(p, r, col);
    }
    for (int i = 0; i < 100; ++i) {  // MainState.cpp:617-638
        float col[3], t[3];
        glibc_uniform3(kColLo, kColHi, col);
        float* v = k.cube(col);
        const float s = glibc_uniform(5.0f, 30.0f);
        rt_cube_scale(v, s, s, s);
        rt_cube_rotate(v, 0.0f, 0.0f, rt_deg_to_rad(glibc_uniform(0.0f, 359.0f)));
        rt_cube_rotate(v, 0.0f, rt_deg_to_rad(glibc_uniform(0.0f, 359.0f)), 0.0f);
        rt_cube_rotate(v, rt_deg_to_rad(glibc_uniform(0.0f, 359.0f)), 0.0f, 0.0f);
        glibc_uniform3(kCubeLo, kCubeHi, t);
        rt_cube_translate(v, t[0], t[1], -t[2]);
    }
}

// SURVEY.md §8d synthetic scene: a portable seeded stream (splitmix64), the
// scene-3 distributions, objects scaled by k.
struct SplitMix {
    uint64_t state;
    uint64_t next() {
        uint64_t z = (state += 0x9E3779B97F4A7C15ull);
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
        return z ^ (z >> 31);
    }
    float uniform(float lo, float hi) {
        const float unit = static_cast<float>(next() >> 40) * (1.0f / 16777216.0f);
        return lo + unit * (hi - lo);
    }
};

}  // namespace

extern "C" {

void rt_cube_init(float vertices[144]) {
    for (int i = 0; i < 36; ++i) {
        const unsigned c = kCorners[i];
        vertices[4 * i + 0] = (c & 1u) ? 1.0f : -1.0f;
        vertices[4 * i + 1] = (c & 2u) ? 1.0f : -1.0f;
        vertices[4 * i + 2] = (c & 4u) ? 1.0f : -1.0f;
        vertices[4 * i + 3] = 1.0f;
    }
}

// Cube.cpp:65-73 with glm scale (matrix_transform.inl:122-134)
void rt_cube_scale(float vertices[144], float sx, float sy, float sz) {
    const Mat4 id = Mat4::identity();
    const float f[3] = {sx, sy, sz};
    Mat4 m;
    for (int j = 0; j < 3; ++j)
        for (int r = 0; r < 4; ++r) m.col[j][r] = id.col[j][r] * f[j];
    for (int r = 0; r < 4; ++r) m.col[3][r] = id.col[3][r];
    transform_all(vertices, m);
}

// Cube.cpp:53-63: rotate(rotate(rotate(I, z, Z), y, Y), x, X)
void rt_cube_rotate(float vertices[144], float rx, float ry, float rz) {
    static const float kZ[3] = {0, 0, 1}, kY[3] = {0, 1, 0}, kX[3] = {1, 0, 0};
    Mat4 m = rotate(Mat4::identity(), rz, kZ);
    m = rotate(m, ry, kY);
    m = rotate(m, rx, kX);
    transform_all(vertices, m);
}

// Cube.cpp:75-83 with glm translate (matrix_transform.inl:40-50)
void rt_cube_translate(float vertices[144], float tx, float ty, float tz) {
    Mat4 m = Mat4::identity();
    for (int r = 0; r < 4; ++r)
        m.col[3][r] = ((m.col[0][r] * tx + m.col[1][r] * ty) + m.col[2][r] * tz) + m.col[3][r];
    transform_all(vertices, m);
}

float rt_deg_to_rad(float degrees) {
    const float pi = 3.1415926535f;  // Utility.h:19
    return degrees * pi / 180.0f;
}

void rt_primary_ray_dir(float out[4]) {
    // glm::perspective(45, 4/3, 0, 100) (matrix_transform.inl:212-231) times
    // (0,0,1,1); only column 2 and 3 survive the zero x, y inputs.
    const float zn = 0.0f, zf = 100.0f;
    Mat4 p{};
    const float th = std::tan(45.0f / 2.0f);
    p.col[0][0] = 1.0f / ((4.0f / 3.0f) * th);
    p.col[1][1] = 1.0f / th;
    p.col[2][2] = -(zf + zn) / (zf - zn);
    p.col[2][3] = -1.0f;
    p.col[3][2] = -(2.0f * zf * zn) / (zf - zn);
    float v[4] = {0.0f, 0.0f, 1.0f, 1.0f};
    p.apply(v);
    std::memcpy(out, v, sizeof v);
}

int rt_scene_reference(int32_t scene_id, uint32_t seed, float* sphere_origins,
                       float* sphere_radius, float* sphere_colours, float* cube_vertices,
                       float* cube_colours, int32_t* num_spheres, int32_t* num_cubes) {
    if (!sphere_origins || !sphere_radius || !sphere_colours || !cube_vertices ||
        !cube_colours || !num_spheres || !num_cubes)
        return RT_ERR_INVALID_ARG;
    Sink k{sphere_origins, sphere_radius, sphere_colours, cube_vertices, cube_colours};
    std::srand(seed);
    switch (scene_id) {
    case 1: build_scene1(k); break;
    case 2: build_scene2(k); break;
    case 3: build_scene3(k); break;
    default: return RT_ERR_INVALID_ARG;
    }
    *num_spheres = k.ns;
    *num_cubes = k.nc;
    return RT_OK;
}

int rt_scene_synthetic(int32_t width, int32_t height, int32_t num_spheres, int32_t num_cubes,
                       uint64_t seed, float k, float* sphere_origins, float* sphere_radius,
                       float* sphere_colours, float* cube_vertices, float* cube_colours) {
    if (width <= 0 || height <= 0 || num_spheres < 0 || num_cubes < 0) return RT_ERR_INVALID_ARG;
    if ((num_spheres && (!sphere_origins || !sphere_radius || !sphere_colours)) ||
        (num_cubes && (!cube_vertices || !cube_colours)))
        return RT_ERR_INVALID_ARG;
    SplitMix rng{seed};
    const float w = static_cast<float>(width), h = static_cast<float>(height);
    for (int32_t i = 0; i < num_spheres; ++i) {
        float* o = sphere_origins + 4 * i;
        o[0] = rng.uniform(0.0f, w);
        o[1] = rng.uniform(0.0f, h);
        o[2] = -rng.uniform(20.0f, 100.0f);
        o[3] = 1.0f;
        sphere_radius[i] = rng.uniform(5.0f, 30.0f) * k;
        float* c = sphere_colours + 4 * i;
        c[0] = rng.uniform(0.05f, 1.0f);
        c[1] = rng.uniform(0.05f, 1.0f);
        c[2] = rng.uniform(0.05f, 1.0f);
        c[3] = 255.0f;
    }
    for (int32_t i = 0; i < num_cubes; ++i) {
        float* c = cube_colours + 4 * i;
        c[0] = rng.uniform(0.05f, 1.0f);
        c[1] = rng.uniform(0.05f, 1.0f);
        c[2] = rng.uniform(0.05f, 1.0f);
        c[3] = 255.0f;
        const float s = rng.uniform(5.0f, 30.0f) * k;
        const float az = rng.uniform(0.0f, 359.0f);
        const float ay = rng.uniform(0.0f, 359.0f);
        const float ax = rng.uniform(0.0f, 359.0f);
        const float tx = rng.uniform(0.0f, w);
        const float ty = rng.uniform(0.0f, h);
        const float tz = -rng.uniform(30.0f, 100.0f);
        float* v = cube_vertices + 144 * i;
        rt_cube_init(v);
        rt_cube_scale(v, s, s, s);
        rt_cube_rotate(v, 0.0f, 0.0f, rt_deg_to_rad(az));
        rt_cube_rotate(v, 0.0f, rt_deg_to_rad(ay), 0.0f);
        rt_cube_rotate(v, rt_deg_to_rad(ax), 0.0f, 0.0f);
        rt_cube_translate(v, tx, ty, tz);
    }
    return RT_OK;
}

void rt_pack_rgba8(const int32_t* frame, int64_t n_pixels, uint32_t* out) {
    for (int64_t i = 0; i < n_pixels; ++i) {
        const int32_t* p = frame + 4 * i;
        out[i] = static_cast<uint32_t>(static_cast<uint8_t>(p[0])) |
                 (static_cast<uint32_t>(static_cast<uint8_t>(p[1])) << 8) |
                 (static_cast<uint32_t>(static_cast<uint8_t>(p[2])) << 16) | 0xFF000000u;
    }
}

uint64_t rt_fnv1a64(const void* words, int64_t n_words, uint64_t basis) {
    const uint32_t* w = static_cast<const uint32_t*>(words);
    uint64_t h = basis;
    for (int64_t i = 0; i < n_words; ++i) h = (h ^ w[i]) * 0x100000001b3ull;
    return h;
}

int rt_abi_version(void) { return RT_ABI_VERSION; }

}  // extern "C"
