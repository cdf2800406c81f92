"""Scene build on the device (include/rt_hip.h
rt_cube_build_device / rt_scene_synthetic_device).

The reference builds cubes on the host through glm, whose rotate takes the
libm's cosf / sinf of a float angle (Cube.cpp:53-63, matrix_transform.inl:
52-58).  The device restates glibc 2.35's sinf / cosf (FMA variant).  CPU
tests check that restatement (host-compiled, the same __host__ __device__
code) against the host libm through the oracle; GPU tests check the device
builds bit for bit against the oracle's cube transforms and synthetic
scenes (orc_cube_*, orc_scene_synthetic, pinned against the reference's own
Cube.cpp in test_oracle.py)."""
import numpy as np
import pytest

F32_MAX = np.float32(3.4028235e38)


def special_floats():
    v = [0.0, -0.0, 1e-45, -1e-45, 1.17549435e-38, 2.0 ** -12, np.nextafter(2.0 ** -12, 0),
         0.78539819, 0.78539813, 0.7853982, 120.0, np.nextafter(np.float32(120.0), 0),
         -120.0, 1e10, -1e10, 1e30, F32_MAX, -F32_MAX, np.pi, -np.pi, np.pi / 2, 2 * np.pi,
         359.0 * 3.1415926535 / 180.0]
    return np.array(v, np.float32)


def float_sample(n_per_exp=2048, seed=5):
    """Floats across every exponent (both signs), random mantissas."""
    rng = np.random.default_rng(seed)
    exps = np.repeat(np.arange(0, 255, dtype=np.uint32), n_per_exp)
    mant = rng.integers(0, 1 << 23, exps.size, dtype=np.uint32)
    sign = rng.integers(0, 2, exps.size, dtype=np.uint32)
    bits = (sign << 31) | (exps << 23) | mant
    return np.concatenate([bits.view(np.float32), special_floats()])


def same_bits(a, b):
    return np.array_equal(np.asarray(a, np.float32).view(np.uint32),
                          np.asarray(b, np.float32).view(np.uint32))


def test_glibc_sincosf_restatement_equals_host_libm(pkg, oracle):
    x = float_sample()
    s, c = pkg.debug_glibc_sincosf(x)
    rs, rc = oracle.libm_sincosf(x)
    assert same_bits(s, rs), np.flatnonzero(s.view(np.uint32) != rs.view(np.uint32))[:10]
    assert same_bits(c, rc), np.flatnonzero(c.view(np.uint32) != rc.view(np.uint32))[:10]


def test_glibc_sincosf_dense_over_scene_angles(pkg, oracle):
    # every float in [0, 2*pi] at a stride: the radian range of the
    # reference's rotate calls (U[0, 359] degrees, MainState.cpp:624-628)
    lo = np.float32(0.0).view(np.uint32)
    hi = np.float32(6.3).view(np.uint32)
    x = np.arange(lo, hi, 97, dtype=np.uint32).view(np.float32)
    s, c = pkg.debug_glibc_sincosf(x)
    rs, rc = oracle.libm_sincosf(x)
    assert same_bits(s, rs) and same_bits(c, rc)


def test_glibc_sincosf_non_finite(pkg):
    s, c = pkg.debug_glibc_sincosf(np.array([np.inf, -np.inf, np.nan], np.float32))
    assert np.isnan(s).all() and np.isnan(c).all()


def test_cube_ops_packing(pkg):
    ops, offsets = pkg.cube_ops([[("scale", 2, 2, 2), ("rotate", 0, 0, 1.0)], [],
                                 [("translate", 1, 2, 3)]])
    assert offsets.tolist() == [0, 2, 2, 3]
    assert ops["op"].tolist() == [1, 2, 3]
    assert ops.dtype.itemsize == 16
    empty_ops, empty_offsets = pkg.cube_ops([])
    assert empty_ops.size == 0 and empty_offsets.tolist() == [0]


def test_device_build_argument_validation(pkg):
    lib = pkg.library()
    assert lib.rt_cube_build_device(None, None, None, 1, None, None, None) == pkg.RT_ERR_INVALID_ARG
    assert lib.rt_scene_synthetic_device(None, 16, 16, 1, 0, 1, 1.0, None, None, None, None,
                                         None, None) == pkg.RT_ERR_INVALID_ARG
    assert lib.rt_selftest_sincosf(None, None, 1, None, None) == pkg.RT_ERR_INVALID_ARG


# ---------------------------------------------------------------------------
# GPU
# ---------------------------------------------------------------------------
# Cubes 1-10 of createScene1/2 (MainState.cpp:434-593) as Cube method calls,
# angles in degrees as the reference writes them (converted per non-zero
# component, MainState.cpp:437 etc.); cube 9's z angle is raw radians (:579).
SCRIPTED = [
    [("s", 40, 40, 40), ("r", 0, 0, 30), ("r", 0, 30, 0), ("t", 70, 60, -60)],
    [("s", 30, 30, 30), ("r", 0, 0, 80), ("r", 0, 250, 0), ("t", 150, 60, -70)],
    [("s", 10, 10, 10), ("r", 0, 0, 160), ("r", 210, 0, 0), ("t", 150, 400, -40)],
    [("s", 50, 50, 50), ("r", 0, 0, 80), ("r", 0, 250, 0), ("t", 450, 200, -80)],
    [("s", 30, 30, 30), ("r", 170, 0, 0), ("r", 0, 150, 0), ("t", 450, 400, -60)],
    [("s", 50, 50, 50), ("r", 0, 0, 80), ("r", 350, 0, 0), ("t", 50, 300, -100)],
    [("s", 70, 70, 70), ("r", 160, 0, 0), ("r", 0, 250, 0), ("t", 530, 300, -100)],
    [("s", 25, 25, 25), ("r", 0, 0, 190), ("r", 0, 140, 0), ("t", 230, 150, -40)],
    [("s", 50, 50, 50), ("r", 0, 130, 0), ("rz_raw", 150, 0, 9.9), ("r", 0, 0, 50),
     ("t", 510, 50, -90)],
    [("s", 24, 24, 24), ("r", 0, 0, 280), ("r", 0, 20, 0), ("t", 350, 340, -40)],
]


def to_radian_program(oracle, steps):
    prog = []
    for op, x, y, z in steps:
        if op == "s":
            prog.append(("scale", x, y, z))
        elif op == "t":
            prog.append(("translate", x, y, z))
        else:
            rad = [oracle.deg2rad(a) if a != 0 else 0.0 for a in (x, y)]
            rz = z if op == "rz_raw" else (oracle.deg2rad(z) if z != 0 else 0.0)
            prog.append(("rotate", rad[0], rad[1], rz))
    return prog


def random_programs(rng, n_cubes):
    programs = []
    for _ in range(n_cubes):
        prog = []
        for _ in range(int(rng.integers(0, 7))):
            kind = rng.integers(0, 3)
            if kind == 0:
                prog.append(("scale", *rng.uniform(-40, 40, 3).astype(np.float32)))
            elif kind == 1:
                r = rng.random()
                span = 6.3 if r < 0.5 else (200.0 if r < 0.8 else 1e6)
                ang = rng.uniform(-span, span, 3).astype(np.float32)
                ang[rng.random(3) < 0.3] = 0.0
                prog.append(("rotate", *ang))
            else:
                prog.append(("translate", *rng.uniform(-1000, 1000, 3).astype(np.float32)))
        programs.append(prog)
    return programs


def build_on_device(pkg, rt, programs, vertices_in=None):
    torch = pytest.importorskip("torch")
    ops, offsets = pkg.cube_ops(programs)
    dev = torch.device("cuda", 0)
    d_ops = torch.from_numpy(ops.view(np.int32).reshape(-1, 4).copy()).to(dev)
    d_off = torch.from_numpy(offsets).to(dev)
    if vertices_in is None:
        d_out = torch.empty((len(programs), 36, 4), dtype=torch.float32, device=dev)
        in_ptr = 0
    else:
        d_out = torch.from_numpy(np.ascontiguousarray(vertices_in, np.float32)).to(dev)
        in_ptr = d_out.data_ptr()  # in place
    rt.cube_build_device(d_ops.data_ptr() if ops.size else 0, d_off.data_ptr(), len(programs),
                         d_out.data_ptr(), in_ptr)
    torch.cuda.synchronize(dev)
    return d_out.cpu().numpy()


@pytest.mark.gpu
def test_device_sincosf_equals_host_libm(pkg, rt, oracle):
    torch = pytest.importorskip("torch")
    dev = torch.device("cuda", 0)
    # every 263rd float of the whole range (16.3M values) plus the samples above
    bits = np.arange(0, 1 << 32, 263, dtype=np.uint64).astype(np.uint32)
    x = np.concatenate([bits.view(np.float32), float_sample()])
    finite = np.isfinite(x)
    d_x = torch.from_numpy(x).to(dev)
    d_s, d_c = torch.empty_like(d_x), torch.empty_like(d_x)
    rt.selftest_sincosf(d_x.data_ptr(), x.size, d_s.data_ptr(), d_c.data_ptr())
    s, c = d_s.cpu().numpy(), d_c.cpu().numpy()
    rs, rc = oracle.libm_sincosf(x)
    assert same_bits(s[finite], rs[finite])
    assert same_bits(c[finite], rc[finite])
    assert np.isnan(s[~finite]).all() and np.isnan(c[~finite]).all()


@pytest.mark.gpu
def test_device_cubes_scripted_scenes(pkg, rt, oracle):
    programs = [to_radian_program(oracle, steps) for steps in SCRIPTED]
    got = build_on_device(pkg, rt, programs)
    want = np.stack([oracle.cube(p) for p in programs])
    assert same_bits(got, want)
    # cubes 1-4 and 1-10 of reference scenes 1 and 2, as the oracle packs them
    assert same_bits(got[:4], oracle.scene_reference(1).cube_vertices)
    assert same_bits(got, oracle.scene_reference(2).cube_vertices)


@pytest.mark.gpu
def test_device_cubes_random_programs(pkg, rt, oracle):
    rng = np.random.default_rng(11)
    programs = random_programs(rng, 3000)
    got = build_on_device(pkg, rt, programs)
    want = np.stack([oracle.cube(p) for p in programs])
    nan = np.isnan(want)
    assert np.array_equal(nan, np.isnan(got))
    assert same_bits(got[~nan], want[~nan])


@pytest.mark.gpu
def test_device_cubes_in_place_animation(pkg, rt, oracle):
    """Re-transform an existing cube set in place (one more rotate and
    translate per frame), as an animated scene would."""
    base_programs = random_programs(np.random.default_rng(3), 200)
    base = np.stack([oracle.cube(p) for p in base_programs])
    step = [[("rotate", 0.01 * i, 0.02, 0.0), ("translate", 1.0, -2.0, 0.5)] for i in range(200)]
    got = build_on_device(pkg, rt, step, vertices_in=base)
    want = np.stack([oracle.cube(p + s) for p, s in zip(base_programs, step)])
    nan = np.isnan(want)
    assert same_bits(got[~nan], want[~nan])


@pytest.mark.gpu
@pytest.mark.parametrize("w,h,n,m,k", [(1920, 1080, 16, 4, 3.0), (4096, 4096, 256, 64, 6.4),
                                       (8192, 8192, 192, 64, 12.8),
                                       (16384, 16384, 4096, 0, 25.6),
                                       (4096, 4096, 20000, 5000, 1.0), (64, 64, 0, 3, 1.0)])
def test_device_synthetic_scene_equals_oracle(pkg, rt, oracle, w, h, n, m, k):
    torch = pytest.importorskip("torch")
    dev = torch.device("cuda", 0)
    d = {"sphere_origins": torch.empty((n, 4), dtype=torch.float32, device=dev),
         "sphere_radius": torch.empty((n,), dtype=torch.float32, device=dev),
         "sphere_colours": torch.empty((n, 4), dtype=torch.float32, device=dev),
         "cube_vertices": torch.empty((m, 36, 4), dtype=torch.float32, device=dev),
         "cube_colours": torch.empty((m, 4), dtype=torch.float32, device=dev)}
    rt.scene_synthetic_device(w, h, n, m, 3, k, {key: t.data_ptr() for key, t in d.items()})
    torch.cuda.synchronize(dev)
    want = oracle.scene_synthetic(w, h, n, m, 3, k)
    for key, t in d.items():
        assert same_bits(t.cpu().numpy(), getattr(want, key)), key


@pytest.mark.gpu
def test_render_from_device_built_scene(pkg, rt, oracle):
    """End to end: build config 2's scene on the device, render it from the
    device arrays, compare the frame with the oracle's."""
    torch = pytest.importorskip("torch")
    dev = torch.device("cuda", 0)
    w, h, n, m = 1920, 1080, 16, 4
    d = {"sphere_origins": torch.empty((n, 4), dtype=torch.float32, device=dev),
         "sphere_radius": torch.empty((n,), dtype=torch.float32, device=dev),
         "sphere_colours": torch.empty((n, 4), dtype=torch.float32, device=dev),
         "cube_vertices": torch.empty((m, 36, 4), dtype=torch.float32, device=dev),
         "cube_colours": torch.empty((m, 4), dtype=torch.float32, device=dev)}
    ptrs = {key: t.data_ptr() for key, t in d.items()}
    rt.scene_synthetic_device(w, h, n, m, 3, 3.0, ptrs)
    out = torch.empty((h, w, 4), dtype=torch.int32, device=dev)
    rt.render_device(dict(ptrs, num_spheres=n, num_cubes=m), w, h, (0, h), out.data_ptr())
    torch.cuda.synchronize(dev)
    s = oracle.scene_synthetic(w, h, n, m, 3, 3.0)
    scene = pkg.Scene(s.sphere_origins, s.sphere_radius, s.sphere_colours, s.cube_vertices,
                      s.cube_colours)
    assert np.array_equal(out.cpu().numpy(), oracle.trace(scene, w, h))
