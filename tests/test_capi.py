"""The C-ABI boundary (include/rt_hip.h): library loads, exports every
declared symbol, and validates arguments without a GPU."""
import ctypes
import re
from pathlib import Path

import numpy as np
import pytest

REPO = Path(__file__).resolve().parents[1]
HEADER = REPO / "include" / "rt_hip.h"
DEBUG_HEADER = REPO / "include" / "rt_hip_debug.h"
DIAG_HEADER = REPO / "include" / "rt_hip_diag.h"


def declared_functions(header=HEADER):
    text = header.read_text()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(rt_[a-z0-9_]+)\s*\(", text)))


def test_header_declares_the_boundary():
    names = declared_functions()
    for required in ("rt_init", "rt_render", "rt_render_device", "rt_destroy",
                     "rt_error_string"):
        assert required in names


def test_library_exports_every_declared_symbol(pkg):
    lib = ctypes.CDLL(str(pkg.library_path()))
    missing = [n for n in declared_functions() if not hasattr(lib, n)]
    assert not missing, missing
    assert set(declared_functions()) == set(pkg.EXPORTED_SYMBOLS)
    hooks = declared_functions(DEBUG_HEADER)
    assert hooks and not [n for n in hooks if not hasattr(lib, n)]


def test_default_build_has_no_diagnostics(pkg):
    """The shipped library (RT_DIAG=0) exports none of the diagnostics
    build's hooks (include/rt_hip_diag.h) and instantiates no ablation
    variant of the trace kernel: only trace3_kernel<0, format>."""
    lib = ctypes.CDLL(str(pkg.library_path()))
    diag = declared_functions(DIAG_HEADER)
    assert "rt_debug_set_trace_mode" in diag
    assert not [n for n in diag if hasattr(lib, n)]
    names = set(re.findall(rb"trace3_kernelILi(\d)ELi(\d)E", pkg.library_path().read_bytes()))
    assert names == {(b"0", b"0"), (b"0", b"1")}, names


def test_abi_version(pkg):
    assert pkg.library().rt_abi_version() == 1


def test_error_strings(pkg):
    lib = pkg.library()
    for code in (0, -1, -2, -3, -4, -5):
        assert lib.rt_error_string(code)
    assert lib.rt_error_string(-99) == b"unknown error"


def test_argument_validation_without_gpu(pkg):
    lib = pkg.library()
    scene = pkg.Scene()
    c = scene.as_c()
    out = np.zeros(16, np.int32)
    d = pkg.primary_ray_dir()
    # NULL context is rejected before any HIP call
    assert lib.rt_render(None, ctypes.byref(c), d.ctypes.data, None, 2, 2, 0, 2, 0,
                         out.ctypes.data, None) == pkg.RT_ERR_INVALID_ARG
    assert lib.rt_render_device(None, ctypes.byref(c), d.ctypes.data, None, 2, 2, 0, 2, 0, 0,
                                out.ctypes.data, None) == pkg.RT_ERR_INVALID_ARG
    assert lib.rt_init(0, None) == pkg.RT_ERR_INVALID_ARG
    assert lib.rt_reserve(None, 640, 480, 1, 1, 0) == pkg.RT_ERR_INVALID_ARG
    k = ctypes.c_int32()
    assert lib.rt_last_kernel(None, ctypes.byref(k)) == pkg.RT_ERR_INVALID_ARG
    # rt_render_multi: no contexts / a NULL context
    ctxs = (ctypes.c_void_p * 2)(None, None)
    assert lib.rt_render_multi(None, 1, ctypes.byref(c), d.ctypes.data, None, 2, 2, 0, 2, 0,
                               out.ctypes.data, None) == pkg.RT_ERR_INVALID_ARG
    assert lib.rt_render_multi(ctxs, 0, ctypes.byref(c), d.ctypes.data, None, 2, 2, 0, 2, 0,
                               out.ctypes.data, None) == pkg.RT_ERR_INVALID_ARG
    assert lib.rt_render_multi(ctxs, 2, ctypes.byref(c), d.ctypes.data, None, 2, 2, 0, 2, 0,
                               out.ctypes.data, None) == pkg.RT_ERR_INVALID_ARG


def test_init_without_gpu_reports_no_device(pkg):
    torch = pytest.importorskip("torch")
    if torch.cuda.is_available():
        pytest.skip("a GPU is present")
    with pytest.raises(pkg.RtError) as e:
        pkg.RayTracer(0)
    assert e.value.status == pkg.RT_ERR_NO_DEVICE


def test_scene_helpers_validate(pkg):
    lib = pkg.library()
    n = ctypes.c_int32()
    assert lib.rt_scene_reference(4, 1, None, None, None, None, None, ctypes.byref(n),
                                  ctypes.byref(n)) == -1
    assert lib.rt_scene_synthetic(0, 10, 1, 1, 1, 1.0, None, None, None, None, None) == -1


def test_fnv1a64_helper_matches_the_fixtures(pkg, oracle):
    """rt_fnv1a64 (the known-answer checksum the bench and the headless driver
    use) equals the oracle's hash of every small fixture frame, and from the
    survey probe's start it gives the reference's recorded known answers."""
    from conftest import PROBE_FNV_BASIS, SURVEY_FNV, load_golden
    for name in ("scene1_640x480", "scene2_640x480", "scene3_640x480", "config1_512x512"):
        g = load_golden(name)
        assert pkg.fnv1a64(g["frame"]) == int(g["fnv1a64"]) == oracle.fnv(g["frame"])
        assert pkg.fnv1a64(pkg.pack_rgba8(g["frame"])) == int(g["fnv1a64_rgba8"])
    for sid in (1, 2, 3):
        g = load_golden(f"scene{sid}_640x480")
        assert pkg.fnv1a64(g["frame"], PROBE_FNV_BASIS) == SURVEY_FNV[sid]
