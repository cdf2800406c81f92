// rt_headless.cpp -- headless C++ host for librt_hip.so.
//
// Stands where the reference's MainState sits (RayTrace/states/MainState.cpp):
// it builds a scene (createScene1/2/3, :419-639, or the synthetic benchmark
// scene), traces it through the C ABI exactly as the rewritten
// MainState::executeRayTracerOpenCL would, prints the
// reference's timing line (:903) and an FNV-1a-64 hash of the int32 frame,
// and can dump the Texture conversion (:974-1045) as a PPM image.
//
//   rt_headless [--scene 1|2|3] [--seed S] [--width W] [--height H]
//               [--synthetic N M k] [--rows A B] [--ppm out.ppm] [--repeat R]
//               [--bands B] [--devices D] [--device-scene]
//               [--format i32x4|rgba8] [--throughput F [--inflight S]]
//               [--known-answer]
//
// --known-answer (reference scene 1, 2 or 3, 640x480, int32x4, the whole
// frame, seed 1): checks the frame against the reference's own CPU frame as
// the survey's probe recorded it (hash above); exit status 1 on a mismatch.
//
// --format rgba8 asks the library for the Texture's pixel format directly
// (RT_FORMAT_RGBA8: one uint32 per pixel, bytes R, G, B, 0xFF -- the
// (uint8_t) wrap and masks of generateImageFromPixels, MainState.cpp:
// 984-994, 1023-1037).  The buffer is what SDL_CreateRGBSurfaceFrom(buf, w,
// h, 32, 4 * w, 0xff, 0xff00, 0xff0000, 0xff000000) wraps without a copy
// (INTEGRATION.md), replacing the per-pixel SDL_FillRect loop; here the PPM
// dump reads it the same way.  The printed hash is FNV-1a-64 over the uint32
// words.
//
// --device-scene (with --synthetic, one band) builds the scene on the GPU
// with rt_scene_synthetic_device, renders it with
// rt_render_device from the device arrays and reads the frame back: no host
// scene build and no scene upload.  The printed hash must equal the host
// build's.
//
// --throughput F [--inflight S] (with --synthetic, one band): the bench's
// frame loop in C++, no Python or torch -- the scene built on the device,
// S (context, stream, device frame) slots used round-robin, each stream
// created with hipExtStreamCreateWithCUMask over every CU so that every
// slot has a hardware queue of its own; untimed frames for
// ~50 ms (the clock ramp), then F frames timed on the host clock between two
// device synchronisations.  Prints us per frame and Grays/s, and the hash of
// every slot's last frame (all must equal the one-frame hash).
//
// --bands splits [A, B) into B row bands traced concurrently through
// rt_render_multi, one rt_ctx per band on device (band % D), each writing its
// rows straight into the shared frame -- the reference's one pixels vector
// (MainState.cpp:676) assembled by disjoint row ranges, SURVEY.md §8(e).
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include <hip/hip_runtime_api.h>

#include "rt_hip.h"

namespace {

// FNV-1a-64 over the frame's 32-bit words (the library's rt_fnv1a64)
uint64_t fnv1a(const int32_t* v, size_t n, uint64_t h = RT_FNV1A64_BASIS) {
    return rt_fnv1a64(v, (int64_t)n, h);
}

// The reference's own CPU frames (MainState::executeRayTracerCPU,
// MainState.cpp:936-956) of scenes 1-3 at 640x480, seed 1, as the survey's
// probe hashed them: FNV-1a-64 over the int32 words from the
// probe's start, 1469598103934665603 (the 64-bit offset basis without its
// last decimal digit).  --known-answer compares against these.
constexpr uint64_t kProbeBasis = 1469598103934665603ull;
constexpr uint64_t kKnownAnswer[3] = {0x57116a151211b387ull, 0xf00fb54672065c63ull,
                                      0xe4eb7bb9d7a1a099ull};

// PPM of a frame in either format: int32x4 pixels take the Texture's
// (uint8_t) wrap (MainState.cpp:1026-1028); RGBA8 words already hold it
// (byte 0 red, 1 green, 2 blue: the surface masks 0xff, 0xff00, 0xff0000).
bool write_ppm(const std::string& path, const std::vector<int32_t>& frame, int w, int h,
               bool rgba8) {
    FILE* f = std::fopen(path.c_str(), "wb");
    if (!f) return false;
    std::fprintf(f, "P6\n%d %d\n255\n", w, h);
    std::vector<unsigned char> row(3 * (size_t)w);
    for (int y = 0; y < h; ++y) {
        for (int x = 0; x < w; ++x) {
            const size_t px = (size_t)y * w + x;
            for (int c = 0; c < 3; ++c)
                row[3 * x + c] =
                    rgba8 ? static_cast<unsigned char>((uint32_t)frame[px] >> (8 * c))
                          : static_cast<unsigned char>(frame[4 * px + c]);
        }
        std::fwrite(row.data(), 1, row.size(), f);
    }
    std::fclose(f);
    return true;
}

struct Band {
    int device = 0, row_begin = 0, row_end = 0;
    rt_ctx* ctx = nullptr;
    rt_timing timing{};
};

// --device-scene: the scene built and rendered on the device, frame read back.
int render_device_scene(Band& band, int width, int height, int row_begin, int row_end, int n,
                        int m, unsigned seed, float k, const float ray_dir[4], int32_t fmt,
                        std::vector<int32_t>& pixels) {
    float *so = nullptr, *sr = nullptr, *sc = nullptr, *cv = nullptr, *cc = nullptr;
    int32_t* out = nullptr;
    const size_t n4 = 4 * sizeof(float) * (size_t)(n > 0 ? n : 1);
    const size_t m4 = 4 * sizeof(float) * (size_t)(m > 0 ? m : 1);
    int status = 1;
    if (hipMalloc(&so, n4) == hipSuccess && hipMalloc(&sr, n4 / 4) == hipSuccess &&
        hipMalloc(&sc, n4) == hipSuccess && hipMalloc(&cv, 36 * m4) == hipSuccess &&
        hipMalloc(&cc, m4) == hipSuccess &&
        hipMalloc(&out, pixels.size() * sizeof(int32_t)) == hipSuccess) {
        int rc = rt_scene_synthetic_device(band.ctx, width, height, n, m, seed, k, so, sr, sc,
                                           cv, cc, nullptr);
        rt_scene scene{so, sr, sc, n, cv, cc, m, nullptr, 0};
        if (rc == RT_OK)
            rc = rt_render_device(band.ctx, &scene, ray_dir, nullptr, width, height, row_begin,
                                  row_end, fmt, RT_PATH_AUTO, out, nullptr);
        if (rc == RT_OK && hipDeviceSynchronize() == hipSuccess &&
            hipMemcpy(pixels.data(), out, pixels.size() * sizeof(int32_t),
                      hipMemcpyDeviceToHost) == hipSuccess) {
            std::printf("device scene: %d spheres, %d cubes built and rendered on the GPU\n",
                        n, m);
            std::printf("frame %dx%d rows [%d,%d) spheres %d cubes %d fnv1a64 %016llx\n",
                        width, height, row_begin, row_end, n, m,
                        (unsigned long long)fnv1a(pixels.data(), pixels.size()));
            status = 0;
        } else {
            std::fprintf(stderr, "device scene render failed: %s\n", rt_error_string(rc));
        }
    } else {
        std::fprintf(stderr, "hipMalloc failed\n");
    }
    for (void* p : {(void*)so, (void*)sr, (void*)sc, (void*)cv, (void*)cc, (void*)out})
        if (p) (void)hipFree(p);
    rt_destroy(band.ctx);
    return status;
}

// --throughput: S slots round-robin over `frames` timed frames.
int throughput(int device, int width, int height, int n, int m, unsigned seed, float k,
               const float ray_dir[4], int32_t fmt, int frames, int slots) {
    if (hipSetDevice(device) != hipSuccess) return 1;
    int n_cu = 0;
    if (hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess)
        return 1;
    std::vector<uint32_t> mask((size_t)(n_cu + 31) / 32, 0u);
    for (int c = 0; c < n_cu; ++c) mask[(size_t)c / 32] |= 1u << (c % 32);
    float *so = nullptr, *sr = nullptr, *sc = nullptr, *cv = nullptr, *cc = nullptr;
    const size_t n4 = 4 * sizeof(float) * (size_t)(n > 0 ? n : 1);
    const size_t m4 = 4 * sizeof(float) * (size_t)(m > 0 ? m : 1);
    const size_t px = (size_t)width * height;
    const size_t frame_words = (fmt == RT_FORMAT_RGBA8 ? 1 : 4) * px;
    std::vector<rt_ctx*> ctx((size_t)slots, nullptr);
    std::vector<hipStream_t> st((size_t)slots, nullptr);
    std::vector<int32_t*> out((size_t)slots, nullptr);
    int status = 1;
    auto fail = [&](const char* what) {
        std::fprintf(stderr, "throughput: %s failed\n", what);
    };
    do {
        if (hipMalloc(&so, n4) != hipSuccess || hipMalloc(&sr, n4 / 4) != hipSuccess ||
            hipMalloc(&sc, n4) != hipSuccess || hipMalloc(&cv, 36 * m4) != hipSuccess ||
            hipMalloc(&cc, m4) != hipSuccess) {
            fail("hipMalloc (scene)");
            break;
        }
        bool ok = true;
        for (int i = 0; i < slots && ok; ++i) {
            ok = rt_init(device, &ctx[(size_t)i]) == RT_OK &&
                 rt_reserve(ctx[(size_t)i], width, height, n, m, fmt) == RT_OK &&
                 hipExtStreamCreateWithCUMask(&st[(size_t)i], (uint32_t)mask.size(),
                                              mask.data()) == hipSuccess &&
                 hipMalloc(&out[(size_t)i], frame_words * sizeof(int32_t)) == hipSuccess;
        }
        if (!ok) {
            fail("slot setup");
            break;
        }
        if (rt_scene_synthetic_device(ctx[0], width, height, n, m, seed, k, so, sr, sc, cv, cc,
                                      nullptr) != RT_OK) {
            fail("rt_scene_synthetic_device");
            break;
        }
        rt_scene scene{so, sr, sc, n, cv, cc, m, nullptr, 0};
        int f = 0;
        auto frame = [&]() {
            const size_t i = (size_t)(f++ % slots);
            return rt_render_device(ctx[i], &scene, ray_dir, nullptr, width, height, 0, height,
                                    fmt, RT_PATH_AUTO, out[i], st[i]);
        };
        using clk = std::chrono::steady_clock;
        // untimed: every slot's first frames, then ~50 ms of load (the clock ramp)
        int rc = RT_OK;
        for (int i = 0; i < 4 * slots && rc == RT_OK; ++i) rc = frame();
        const auto r0 = clk::now();
        while (rc == RT_OK && clk::now() - r0 < std::chrono::milliseconds(50)) {
            for (int i = 0; i < 16 && rc == RT_OK; ++i) rc = frame();
            if (hipDeviceSynchronize() != hipSuccess) rc = RT_ERR_HIP;
        }
        if (rc != RT_OK || hipDeviceSynchronize() != hipSuccess) {
            fail("warm-up frames");
            break;
        }
        f = 0;
        const auto t0 = clk::now();
        for (int i = 0; i < frames && rc == RT_OK; ++i) rc = frame();
        if (rc != RT_OK || hipDeviceSynchronize() != hipSuccess) {
            fail("timed frames");
            break;
        }
        const double us = std::chrono::duration<double, std::micro>(clk::now() - t0).count() /
                          frames;
        std::vector<int32_t> host(frame_words);
        std::printf("throughput %dx%d spheres %d cubes %d %s: %d frames, %d in flight: "
                    "%.2f us per frame, %.1f Grays/s\n",
                    width, height, n, m, fmt == RT_FORMAT_RGBA8 ? "rgba8" : "i32x4", frames,
                    slots, us, (double)px / us / 1e3);
        ok = true;
        for (int i = 0; i < slots && ok; ++i) {
            ok = hipMemcpy(host.data(), out[(size_t)i], frame_words * sizeof(int32_t),
                           hipMemcpyDeviceToHost) == hipSuccess;
            if (ok)
                std::printf("slot %d fnv1a64 %016llx\n", i,
                            (unsigned long long)fnv1a(host.data(), host.size()));
        }
        int32_t kern = 0;
        (void)rt_last_kernel(ctx[0], &kern);
        std::printf("kernel %d\n", (int)kern);
        status = ok ? 0 : 1;
    } while (false);
    (void)hipDeviceSynchronize();
    for (int i = 0; i < slots; ++i) {
        if (out[(size_t)i]) (void)hipFree(out[(size_t)i]);
        if (st[(size_t)i]) (void)hipStreamDestroy(st[(size_t)i]);
        rt_destroy(ctx[(size_t)i]);
    }
    for (void* p : {(void*)so, (void*)sr, (void*)sc, (void*)cv, (void*)cc})
        if (p) (void)hipFree(p);
    return status;
}

}  // namespace

int main(int argc, char** argv) {
    int scene_id = 1, width = 640, height = 480, repeat = 1;
    unsigned seed = 1;
    int syn_n = -1, syn_m = -1;
    float syn_k = 1.0f;
    int row_begin = 0, row_end = -1;
    int n_bands = 1, n_devices = 1;
    bool device_scene = false;
    int tp_frames = 0, tp_slots = 2;
    int32_t fmt = RT_FORMAT_I32X4;
    bool known_answer = false;
    std::string ppm;
    for (int i = 1; i < argc; ++i) {
        std::string a = argv[i];
        auto next = [&](void) -> const char* {
            if (i + 1 >= argc) {
                std::fprintf(stderr, "missing value for %s\n", a.c_str());
                std::exit(2);
            }
            return argv[++i];
        };
        if (a == "--scene") scene_id = std::atoi(next());
        else if (a == "--seed") seed = (unsigned)std::strtoul(next(), nullptr, 10);
        else if (a == "--width") width = std::atoi(next());
        else if (a == "--height") height = std::atoi(next());
        else if (a == "--synthetic") {
            syn_n = std::atoi(next());
            syn_m = std::atoi(next());
            syn_k = (float)std::atof(next());
        } else if (a == "--rows") {
            row_begin = std::atoi(next());
            row_end = std::atoi(next());
        } else if (a == "--ppm") ppm = next();
        else if (a == "--repeat") repeat = std::atoi(next());
        else if (a == "--bands") n_bands = std::atoi(next());
        else if (a == "--devices") n_devices = std::atoi(next());
        else if (a == "--device-scene") device_scene = true;
        else if (a == "--known-answer") known_answer = true;
        else if (a == "--throughput") tp_frames = std::atoi(next());
        else if (a == "--inflight") tp_slots = std::atoi(next());
        else if (a == "--format") {
            const std::string v = next();
            if (v == "i32x4") fmt = RT_FORMAT_I32X4;
            else if (v == "rgba8") fmt = RT_FORMAT_RGBA8;
            else {
                std::fprintf(stderr, "--format takes i32x4 or rgba8\n");
                return 2;
            }
        }
        else {
            std::fprintf(stderr, "unknown option %s\n", a.c_str());
            return 2;
        }
    }
    if (row_end < 0) row_end = height;
    if (n_bands < 1 || n_devices < 1 || row_begin < 0 || row_end > height ||
        row_begin >= row_end) {
        std::fprintf(stderr, "bad --rows/--bands/--devices\n");
        return 2;
    }
    if (known_answer && (syn_n >= 0 || scene_id < 1 || scene_id > 3 || seed != 1 ||
                         width != 640 || height != 480 || row_begin != 0 || row_end != height ||
                         fmt != RT_FORMAT_I32X4)) {
        std::fprintf(stderr, "--known-answer needs --scene 1|2|3 at 640x480, seed 1, int32x4, "
                             "the whole frame\n");
        return 2;
    }
    if (device_scene && (syn_n < 0 || n_bands != 1)) {
        std::fprintf(stderr, "--device-scene needs --synthetic and one band\n");
        return 2;
    }
    if (tp_frames > 0) {
        if (syn_n < 0 || n_bands != 1 || tp_slots < 1 || tp_slots > 8 || row_begin != 0 ||
            row_end != height) {
            std::fprintf(stderr, "--throughput needs --synthetic, the whole frame, one band and "
                                 "1..8 --inflight slots\n");
            return 2;
        }
        float d[4];
        rt_primary_ray_dir(d);
        return throughput(0, width, height, syn_n, syn_m, seed, syn_k, d, fmt, tp_frames,
                          tp_slots);
    }

    // Scene vectors, MainState.h:99-106 (cubes already flattened, :646-655).
    const int cap_s = syn_n >= 0 ? syn_n : 100, cap_c = syn_m >= 0 ? syn_m : 100;
    std::vector<float> so(4 * (size_t)cap_s), sr((size_t)cap_s), sc(4 * (size_t)cap_s);
    std::vector<float> cv(144 * (size_t)cap_c), cc(4 * (size_t)cap_c);
    int32_t ns = 0, nc = 0;
    int rc;
    if (syn_n >= 0) {
        rc = rt_scene_synthetic(width, height, syn_n, syn_m, seed, syn_k, so.data(), sr.data(),
                                sc.data(), cv.data(), cc.data());
        ns = syn_n;
        nc = syn_m;
    } else {
        rc = rt_scene_reference(scene_id, seed, so.data(), sr.data(), sc.data(), cv.data(),
                                cc.data(), &ns, &nc);
    }
    if (rc != RT_OK) {
        std::fprintf(stderr, "scene construction failed: %s\n", rt_error_string(rc));
        return 1;
    }

    // One context per band: MainState ctor -> openCLInit (:52).
    const int rows = row_end - row_begin;
    if (n_bands > rows) n_bands = rows;
    std::vector<Band> bands(n_bands);
    for (int b = 0; b < n_bands; ++b) {
        Band& band = bands[b];
        band.device = b % n_devices;
        band.row_begin = row_begin + (int)((int64_t)rows * b / n_bands);
        band.row_end = row_begin + (int)((int64_t)rows * (b + 1) / n_bands);
        rc = rt_init(band.device, &band.ctx);
        // the rest of openCLInit's one-time work, for this band's frame
        if (rc == RT_OK)
            rc = rt_reserve(band.ctx, width, band.row_end - band.row_begin, ns, nc, fmt);
        if (rc != RT_OK) {
            std::fprintf(stderr, "rt_init / rt_reserve(%d) failed: %s\n", band.device,
                         rt_error_string(rc));
            for (Band& o : bands) rt_destroy(o.ctx);
            return 1;
        }
    }
    float ray_dir[4];
    rt_primary_ray_dir(ray_dir);  // (0,0,-1,-1), MainState.cpp:37-39
    rt_scene scene{so.data(), sr.data(), sc.data(), ns, cv.data(), cc.data(), nc, nullptr, 0};
    // MainState::pixels (MainState.h:86, reserved at :215): 4 ints per pixel,
    // or the Texture's one RGBA8 word per pixel
    const bool rgba8 = fmt == RT_FORMAT_RGBA8;
    std::vector<int32_t> pixels((rgba8 ? 1 : 4) * (size_t)width * rows);
    if (device_scene) return render_device_scene(bands[0], width, height, row_begin, row_end,
                                                 syn_n, syn_m, seed, syn_k, ray_dir, fmt, pixels);
    // rt_render_multi: one host thread and one context per band, each band's
    // rows written straight into `pixels` (same row split as `bands`)
    std::vector<rt_ctx*> ctxs;
    for (Band& band : bands) ctxs.push_back(band.ctx);
    std::vector<rt_timing> timings((size_t)n_bands);
    int status = 0;
    for (int r = 0; r < repeat && status == 0; ++r) {
        std::printf("HIP Ray Tracer Begin\n");
        rc = rt_render_multi(ctxs.data(), n_bands, &scene, ray_dir, nullptr, width, height,
                             row_begin, row_end, fmt, pixels.data(), timings.data());
        if (rc != RT_OK) {
            std::fprintf(stderr, "rt_render_multi failed: %s\n", rt_error_string(rc));
            status = 1;
            break;
        }
        for (int b = 0; b < n_bands; ++b) {
            Band& band = bands[b];
            band.timing = timings[(size_t)b];
            const rt_timing& t = band.timing;
            std::printf("Time Taken: %.0f microseconds (upload %.1f, kernels %.1f, readback %.1f; "
                        "%s path)",
                        t.total_us, t.upload_us, t.kernel_us, t.download_us,
                        t.path == RT_PATH_BINNED ? "binned" : "generic");
            if (n_bands > 1)
                std::printf(" band %d rows [%d,%d) device %d", b, band.row_begin, band.row_end,
                            band.device);
            std::printf("\n");
        }
    }
    if (status == 0) {
        std::printf("frame %dx%d rows [%d,%d) spheres %d cubes %d %s fnv1a64 %016llx\n", width,
                    height, row_begin, row_end, ns, nc, rgba8 ? "rgba8" : "i32x4",
                    (unsigned long long)fnv1a(pixels.data(), pixels.size()));
        if (!ppm.empty() && !write_ppm(ppm, pixels, width, rows, rgba8))
            std::fprintf(stderr, "could not write %s\n", ppm.c_str());
        if (known_answer) {
            const uint64_t got = fnv1a(pixels.data(), pixels.size(), kProbeBasis);
            const uint64_t want = kKnownAnswer[scene_id - 1];
            std::printf("known answer scene %d: %016llx, reference CPU frame %016llx: %s\n",
                        scene_id, (unsigned long long)got, (unsigned long long)want,
                        got == want ? "match" : "MISMATCH");
            if (got != want) status = 1;
        }
    }
    for (Band& band : bands) rt_destroy(band.ctx);
    return status;
}
