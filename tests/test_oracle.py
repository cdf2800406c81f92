"""The oracle (oracle/rt_oracle.c) pinned against the reference.

Pins (SURVEY.md §0 F5/F7 and §8c recorded them from the reference's own
executeRayTracerCPU, MainState.cpp:936-972, built and run in the survey's
probe):
  * the probe's FNV-1a-64 known answers for scenes 1-3 @640x480
    (57116a151211b387 / f00fb54672065c63 / e4eb7bb9d7a1a099): reproduced
    bit for bit by the oracle's frames once the hash starts from
    1469598103934665603 -- the 64-bit FNV offset basis 14695981039346656037
    with its last decimal digit dropped.  That start was found, not guessed:
    running FNV-1a backwards (x -> x * P^-1 ^ word) from each known answer
    over the oracle's frame gives the same state before the first word for
    all three scenes, and that state is this number;
  * scene 1 @640x480: 38,285 lit pixels, max channel 257, 6 pixels > 255, min 0;
  * CPU vs the reference's own fp32 OpenCL kernel (rayTracer.cl): 33 pixels
    differ in scenes 1 and 2 (max channel difference 205 in scene 1), 0 in
    scene 3 -- reproduced here only with right-to-left evaluation of the
    Random::getFloat() constructor arguments, which is what pins that order;
  * cube packing: the reference's unmodified Cube.cpp (oracle/_ref).
"""
from pathlib import Path

import numpy as np
import pytest

from conftest import (FNV_PRIME, PROBE_FNV_BASIS, SURVEY_FNV, SURVEY_FNV_FMA, Oracle,
                      load_golden, probe_fnv)
from oracle_lib import ref_cube, ref_cube_lib

RAY_DIR = np.array([0.0, 0.0, -1.0, -1.0], np.float32)


def test_primary_ray_dir(oracle):
    """perspective(45, 4/3, 0, 100) * (0,0,1,1) is exactly (0,0,-1,-1)."""
    assert np.array_equal(oracle.ray_dir(), RAY_DIR)


def _fnv_state_before(frame, h_end):
    """Run FNV-1a backwards over `frame` from the final hash h_end: the state
    the hash must have had before the frame's first word."""
    inv = pow(FNV_PRIME, -1, 1 << 64)
    h = h_end
    for w in reversed(np.ascontiguousarray(frame, np.int32).ravel().view(np.uint32).tolist()):
        h = ((h * inv) & 0xFFFFFFFFFFFFFFFF) ^ w
    return h


@pytest.mark.parametrize("scene_id", [1, 2, 3])
def test_survey_known_answers(oracle, scene_id):
    """The reference's own CPU frames (the survey probe's hashes of
    executeRayTracerCPU's `pixels`, MainState.cpp:936-956) equal the oracle's
    bit for bit: every one of the 1,228,800 int32 words enters the hash."""
    frame = oracle.trace(oracle.scene_reference(scene_id, 1, rtl=1), 640, 480, threads=4)
    assert probe_fnv(frame) == SURVEY_FNV[scene_id]
    # how the start was found: the backwards run lands on it for every scene
    assert _fnv_state_before(frame, SURVEY_FNV[scene_id]) == PROBE_FNV_BASIS
    assert PROBE_FNV_BASIS == 14695981039346656037 // 10
    # the committed fixture is the same frame
    assert np.array_equal(frame, load_golden(f"scene{scene_id}_640x480")["frame"])


def _cpu_has_fma():
    try:
        flags = Path("/proc/cpuinfo").read_text()
    except OSError:
        return False
    return " fma " in flags and " avx2 " in flags


@pytest.mark.skipif(not _cpu_has_fma(), reason="the FMA variant needs an x86-64-v3 CPU")
@pytest.mark.parametrize("scene_id", [1, 2, 3])
def test_survey_fma_known_answers(scene_id):
    """The probe's -march=native hashes (scenes 1 and 2
    change under FMA, scene 3 does not) from the oracle's own source built
    with FMA contraction (liboracle_fma.so): GCC fuses a multiply into an add
    only where one expression holds both, so these match only if the
    restatement writes the reference's expressions -- glm's rotate and dot,
    the Moller-Trumbore macros, the sphere test, the shade -- as the
    reference does at every such point."""
    fo = Oracle(fma=True)
    frame = fo.trace(fo.scene_reference(scene_id, 1, rtl=1), 640, 480, threads=4)
    assert probe_fnv(frame) == SURVEY_FNV_FMA[scene_id]


def test_survey_known_answers_are_frame_sensitive(oracle):
    """Negative control: one channel of one pixel off by one, or the other
    evaluation order of the scene's random numbers, no longer gives the
    survey's hash."""
    frame = oracle.trace(oracle.scene_reference(1), 640, 480, threads=4)
    bad = frame.copy()
    bad[240, 320, 0] += 1
    assert probe_fnv(bad) != SURVEY_FNV[1]
    ltr = oracle.trace(oracle.scene_reference(2, 1, rtl=0), 640, 480, threads=4)
    assert probe_fnv(ltr) != SURVEY_FNV[2]


def test_scene1_statistics_pin(oracle):
    frame = oracle.trace(oracle.scene_reference(1), 640, 480)
    assert frame.min() == 0 and frame.max() == 257
    assert int((frame[..., :3].sum(-1) != 0).sum()) == 38285
    assert int((frame[..., :3] > 255).any(-1).sum()) == 6
    assert (frame[..., 3] == 255).all()


@pytest.mark.parametrize("scene_id,n_diff,max_diff", [(1, 33, 205), (2, 33, None), (3, 0, 0)])
def test_cpu_vs_opencl_kernel_divergence_pin(oracle, scene_id, n_diff, max_diff):
    sc = oracle.scene_reference(scene_id, 1, rtl=1)
    cpu = oracle.trace(sc, 640, 480, threads=4)
    cl = oracle.trace_cl32(sc, 640, 480)
    diff = (cpu != cl).any(-1)
    assert int(diff.sum()) == n_diff
    if max_diff is not None:
        assert int(np.abs(cpu - cl).max()) == max_diff


def test_argument_order_is_right_to_left(oracle):
    """Left-to-right evaluation would give scene 3 a CPU/kernel divergence the
    survey's probe did not see."""
    sc = oracle.scene_reference(3, 1, rtl=0)
    cpu = oracle.trace(sc, 640, 480, threads=4)
    assert int((cpu != oracle.trace_cl32(sc, 640, 480)).any(-1).sum()) != 0


@pytest.mark.parametrize("name", ["scene1_640x480", "scene2_640x480", "scene3_640x480",
                                  "config1_512x512", "config2_1920x1080",
                                  "config2s_1920x1080"])
def test_golden_fixture_reproduces(oracle, name):
    g = load_golden(name)
    from types import SimpleNamespace
    sc = SimpleNamespace(**{k: g[k] for k in ("sphere_origins", "sphere_radius",
                                              "sphere_colours", "cube_vertices", "cube_colours")})
    frame = oracle.trace(sc, int(g["width"]), int(g["height"]), ray_dir=g["ray_dir"], threads=8)
    assert np.array_equal(frame, g["frame"])
    assert oracle.fnv(frame) == int(g["fnv1a64"])


@pytest.mark.parametrize("scene_id", [1, 2, 3])
def test_reference_scene_fixture_arrays(oracle, scene_id):
    """The committed scene arrays are the oracle's scene construction (glibc
    rand/cosf on this image); a libc change would show up here."""
    g = load_golden(f"scene{scene_id}_640x480")
    sc = oracle.scene_reference(scene_id, 1)
    for k in ("sphere_origins", "sphere_radius", "sphere_colours", "cube_vertices",
              "cube_colours"):
        assert np.array_equal(getattr(sc, k).view(np.uint32), g[k].view(np.uint32)), k


def _random_ops(rng, n):
    ops = []
    for _ in range(n):
        kind = rng.choice(["scale", "rotate", "translate"])
        if kind == "scale":
            ops.append(("scale", *rng.uniform(0.01, 80, 3)))
        elif kind == "rotate":
            ops.append(("rotate", *rng.uniform(-7, 7, 3)))
        else:
            ops.append(("translate", *rng.uniform(-700, 700, 3)))
    return ops


@pytest.fixture(scope="module")
def refcube():
    lib = ref_cube_lib()
    if lib is None:
        pytest.skip("oracle/_ref not built (needs /root/reference)")
    return lib


def test_cube_packing_vs_reference_cube_cpp(oracle, refcube):
    rng = np.random.default_rng(5)
    for _ in range(300):
        ops = _random_ops(rng, int(rng.integers(1, 6)))
        want, col = ref_cube(refcube, (0.3, 0.6, 0.9, 255.0), ops)
        got = oracle.cube(ops)
        assert np.array_equal(got.view(np.uint32), want.view(np.uint32)), ops
        assert np.array_equal(col, np.float32([0.3, 0.6, 0.9, 255.0]))


def test_reference_scene_cubes_vs_reference_cube_cpp(oracle, refcube):
    """Scene 1's four hand-placed cubes (MainState.cpp:434-461) through the
    reference's own Cube.cpp."""
    d = oracle.deg2rad
    specs = [((1, 1, 0, 255), [("scale", 40, 40, 40), ("rotate", 0, 0, d(30)),
                               ("rotate", 0, d(30), 0), ("translate", 70, 60, -60)]),
             ((0, 1, 1, 255), [("scale", 30, 30, 30), ("rotate", 0, 0, d(80)),
                               ("rotate", 0, d(250), 0), ("translate", 150, 60, -70)]),
             ((0, 0, 1, 255), [("scale", 10, 10, 10), ("rotate", 0, 0, d(160)),
                               ("rotate", d(210), 0, 0), ("translate", 150, 400, -40)]),
             ((1, 0, 0, 255), [("scale", 50, 50, 50), ("rotate", 0, 0, d(80)),
                               ("rotate", 0, d(250), 0), ("translate", 450, 200, -80)])]
    sc = oracle.scene_reference(1)
    for i, (col, ops) in enumerate(specs):
        want, c = ref_cube(refcube, col, ops)
        assert np.array_equal(sc.cube_vertices[i].view(np.uint32), want.view(np.uint32))
        assert np.array_equal(sc.cube_colours[i], c)


def test_intersect_sphere_semantics(oracle):
    o = np.float32([10, 10, 0, 1])
    # tca < 0: sphere in front of the origin plane never hits (MainState.cpp:305)
    assert oracle.intersect_sphere(o, RAY_DIR, 5.0, [10, 10, 20, 1]) == 0.0
    # origin inside the sphere: t0 < 0 is returned (no t > 0 test)
    assert oracle.intersect_sphere(o, RAY_DIR, 30.0, [10, 10, -10, 1]) < 0
    assert oracle.intersect_sphere(o, RAY_DIR, 5.0, [10, 10, -50, 1]) == 45.0


def test_intersect_tri_no_t_positive_test(oracle):
    """Triangles behind the ray origin are accepted (t < 0), F7."""
    hit, t = oracle.intersect_tri([0, 0, 0], [0, 0, -1], [-5, -5, 10], [5, -5, 10], [0, 5, 10])
    assert hit == 1 and t == -10.0
    hit, _ = oracle.intersect_tri([0, 0, 0], [0, 0, -1], [-5, -5, 0], [5, -5, 0], [10, -5, 0])
    assert hit == 0  # degenerate: det == 0


def test_get_float_vs_reference_random_cpp(oracle):
    """The scenes' random numbers (Random::init + Random::getFloat,
    Random.cpp:10-42) against the reference's own Random.cpp compiled
    unmodified (oracle/_ref/libref_random.so): same glibc rand() stream,
    bit-identical floats, over the ranges createScene2/3 use."""
    from oracle_lib import ref_random_lib
    ref = ref_random_lib()
    if ref is None:
        pytest.skip("oracle/_ref not built (needs /root/reference)")
    ranges = [(0.0, 630.0), (0.0, 470.0), (20.0, 100.0), (5.0, 30.0), (0.05, 1.0),
              (0.0, 359.0), (30.0, 100.0), (-7.0, 7.0)]
    for seed in (1, 2, 7, 12345):
        ref.ref_random_init(seed)
        want = [ref.ref_random_get_float(*ranges[i % len(ranges)]) for i in range(4000)]
        oracle.lib.orc_srand(seed)
        got = [oracle.lib.orc_get_float(*ranges[i % len(ranges)]) for i in range(4000)]
        assert np.array_equal(np.float32(got), np.float32(want)), seed


def test_glm_arithmetic_vs_reference_glm(oracle):
    """The oracle's glm restatements against the reference's vendored glm
    0.9.6 (oracle/_ref/libref_glm.so): the primary ray direction
    (MainState.cpp:37-39) and the sphere test's vec4 arithmetic
    (MainState.cpp:300-327, glm::dot pairwise order), bit for bit."""
    import ctypes
    from oracle_lib import ref_glm_lib
    ref = ref_glm_lib()
    if ref is None:
        pytest.skip("oracle/_ref not built (needs /root/reference)")
    d = np.zeros(4, np.float32)
    ref.ref_glm_ray_dir(d.ctypes.data)
    assert np.array_equal(d.view(np.uint32), oracle.ray_dir().view(np.uint32))
    rng = np.random.default_rng(17)
    dirs = [RAY_DIR] + [rng.uniform(-1, 1, 4).astype(np.float32) for _ in range(3)]
    n_hits = 0
    for i in range(20000):
        o = np.float32([rng.uniform(-50, 700), rng.uniform(-50, 500), rng.uniform(-5, 5), 1.0])
        c = np.float32([rng.uniform(-50, 700), rng.uniform(-50, 500), -rng.uniform(0, 120),
                        [1.0, 0.5, 3.0][i % 3]])
        if i % 4 == 0:  # near-tangent: centre just off the ray through o
            c[:2] = o[:2] + np.float32(rng.uniform(-3, 3, 2))
        r = np.float32(rng.uniform(0.5, 60.0))
        dv = np.ascontiguousarray(dirs[i % len(dirs)])
        want = ref.ref_glm_sphere(o.ctypes.data, dv.ctypes.data, ctypes.c_float(r), c.ctypes.data)
        got = oracle.intersect_sphere(o, dv, float(r), c)
        assert np.float32(got).view(np.uint32) == np.float32(want).view(np.uint32), (o, c, r, dv)
        n_hits += want != 0.0
    assert n_hits > 1000
    for _ in range(2000):
        a, b = rng.uniform(-1e3, 1e3, (2, 4)).astype(np.float32)
        want = ref.ref_glm_dot4(a.ctypes.data, b.ctypes.data)
        got = ((a[0] * b[0]) + (a[1] * b[1])) + ((a[2] * b[2]) + (a[3] * b[3]))
        assert np.float32(got) == np.float32(want)
