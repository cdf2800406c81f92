"""opencl-ray-tracer_amd -- Python host mirror of the MI355X ray tracer's C ABI.

The product is ``librt_hip.so`` (``csrc/``, declared in ``include/rt_hip.h``):
the HIP kernels plus the C ABI that replaces the reference's OpenCL dispatch
``MainState::executeRayTracerOpenCL`` (RayTrace/states/MainState.cpp:641-934).
This module binds that library with ctypes and mirrors the reference's
call-site vocabulary (``MainState`` with ``createScene1..3`` and
``executeRayTracer``), so tests and the benchmark read like the reference's
own control flow.  There is no CPU fallback here: if the library or a GPU is
missing, calls raise.
"""
from __future__ import annotations

import ctypes
import os
from dataclasses import dataclass, field
from pathlib import Path
from typing import Optional, Tuple

import numpy as np

__all__ = [
    "RT_OK", "RT_ERR_INVALID_ARG", "RT_ERR_NO_DEVICE", "RT_ERR_HIP", "RT_ERR_OUT_OF_MEMORY",
    "RT_ERR_UNSUPPORTED", "RT_FORMAT_I32X4", "RT_FORMAT_RGBA8", "RT_PATH_AUTO", "RT_PATH_BINNED",
    "RT_PATH_GENERIC", "RtError", "Scene", "Timing", "RayTracer", "MainState",
    "library", "library_path", "primary_ray_dir", "pack_rgba8", "cube_packed",
    "deg_to_rad", "encode_png", "EXPORTED_SYMBOLS", "CUBE_OP_DTYPE", "cube_ops", "render_multi",
    "debug_glibc_sincosf", "host_register", "host_unregister",
]

PKG_DIR = Path(__file__).resolve().parent
RT_OK = 0
RT_ERR_INVALID_ARG, RT_ERR_NO_DEVICE, RT_ERR_HIP = -1, -2, -3
RT_ERR_OUT_OF_MEMORY, RT_ERR_UNSUPPORTED = -4, -5
RT_FORMAT_I32X4, RT_FORMAT_RGBA8 = 0, 1
RT_PATH_AUTO, RT_PATH_BINNED, RT_PATH_GENERIC = 0, 1, 2
_FORMATS = {"i32x4": RT_FORMAT_I32X4, "rgba8": RT_FORMAT_RGBA8}
_PATHS = {"auto": RT_PATH_AUTO, "binned": RT_PATH_BINNED, "generic": RT_PATH_GENERIC}

# Every symbol include/rt_hip.h declares (tests check the .so exports them).
EXPORTED_SYMBOLS = (
    "rt_init", "rt_destroy", "rt_error_string", "rt_render", "rt_render_path",
    "rt_render_device", "rt_profile_enable", "rt_profile_read", "rt_device_info",
    "rt_cube_init", "rt_cube_scale", "rt_cube_rotate", "rt_cube_translate",
    "rt_deg_to_rad", "rt_primary_ray_dir", "rt_scene_reference", "rt_scene_synthetic",
    "rt_pack_rgba8", "rt_abi_version", "rt_cube_build_device", "rt_scene_synthetic_device",
    "rt_render_multi", "rt_shared_alloc", "rt_shared_open", "rt_shared_close", "rt_shared_free",
    "rt_host_register", "rt_host_unregister", "rt_reserve", "rt_last_kernel", "rt_fnv1a64",
)
# rt_last_kernel's codes (RT_KERNEL_*, rt_hip.h) by name
KERNEL_NAMES = {0: None, 1: "trace3_kernel", 2: "trace_small_kernel", 3: "frame_small_kernel",
                4: "generic_kernel", 5: "trace3_split_kernel", 6: "trace_bin_kernel"}
# exported only by the diagnostics build (make RT_DIAG=1, include/rt_hip_diag.h)
DIAG_SYMBOLS = ("rt_debug_set_trace_mode",)


class RtError(RuntimeError):
    """A negative status from librt_hip.so (rt_error_string text attached)."""

    def __init__(self, status: int, what: str):
        self.status = status
        super().__init__(f"{what}: {_error_string(status)} ({status})")


class _Scene(ctypes.Structure):
    _fields_ = [
        ("sphere_origins", ctypes.c_void_p), ("sphere_radius", ctypes.c_void_p),
        ("sphere_colours", ctypes.c_void_p), ("num_spheres", ctypes.c_int32),
        ("cube_vertices", ctypes.c_void_p), ("cube_colours", ctypes.c_void_p),
        ("num_cubes", ctypes.c_int32), ("lights", ctypes.c_void_p),
        ("num_lights", ctypes.c_int32),
    ]


class _Timing(ctypes.Structure):
    _fields_ = [
        ("total_us", ctypes.c_double), ("upload_us", ctypes.c_double),
        ("kernel_us", ctypes.c_double), ("download_us", ctypes.c_double),
        ("path", ctypes.c_int32),
    ]


class _IpcHandle(ctypes.Structure):
    _fields_ = [("bytes", ctypes.c_ubyte * 64)]


_LIB: Optional[ctypes.CDLL] = None


def library_path() -> Path:
    return Path(os.environ.get("RT_HIP_LIBRARY", PKG_DIR / "librt_hip.so"))


def library() -> ctypes.CDLL:
    """Load librt_hip.so (built by ``make -C csrc`` / ``__graft_entry__.build``)."""
    global _LIB
    if _LIB is not None:
        return _LIB
    path = library_path()
    if not path.exists():
        raise RuntimeError(f"{path} is missing: build it with `make -C {PKG_DIR / 'csrc'}`")
    # One HIP runtime per process: PyTorch-ROCm ships its own libamdhip64.so.7
    # (same SONAME as /opt/rocm's).  Whichever is loaded first serves every
    # later user, and torch cannot run on a runtime other than its own, so
    # load torch's first when torch is installed (RT_NO_TORCH=1 opts out).
    if os.environ.get("RT_NO_TORCH", "0") != "1":
        try:
            import torch  # noqa: F401  (plumbing: device memory, streams, RCCL)
        except ImportError:
            pass
    lib = ctypes.CDLL(str(path))
    vp, i32, f32 = ctypes.c_void_p, ctypes.c_int32, ctypes.c_float
    sig = {
        "rt_init": (ctypes.c_int, [ctypes.c_int, ctypes.POINTER(vp)]),
        "rt_destroy": (None, [vp]),
        "rt_error_string": (ctypes.c_char_p, [ctypes.c_int]),
        "rt_render": (ctypes.c_int, [vp, ctypes.POINTER(_Scene), vp, vp, i32, i32, i32, i32,
                                     i32, vp, ctypes.POINTER(_Timing)]),
        "rt_render_path": (ctypes.c_int, [vp, ctypes.POINTER(_Scene), vp, vp, i32, i32, i32,
                                          i32, i32, i32, vp, ctypes.POINTER(_Timing)]),
        "rt_render_device": (ctypes.c_int, [vp, ctypes.POINTER(_Scene), vp, vp, i32, i32, i32,
                                            i32, i32, i32, vp, vp]),
        "rt_render_multi": (ctypes.c_int, [ctypes.POINTER(vp), i32, ctypes.POINTER(_Scene), vp,
                                           vp, i32, i32, i32, i32, i32, vp,
                                           ctypes.POINTER(_Timing)]),
        "rt_shared_alloc": (ctypes.c_int, [vp, ctypes.c_int64, ctypes.POINTER(vp),
                                           ctypes.POINTER(_IpcHandle)]),
        "rt_shared_open": (ctypes.c_int, [vp, ctypes.POINTER(_IpcHandle), ctypes.POINTER(vp)]),
        "rt_shared_close": (ctypes.c_int, [vp, vp]),
        "rt_shared_free": (ctypes.c_int, [vp, vp]),
        "rt_host_register": (ctypes.c_int, [vp, ctypes.c_int64]),
        "rt_host_unregister": (ctypes.c_int, [vp]),
        "rt_profile_enable": (ctypes.c_int, [vp, ctypes.c_int]),
        "rt_profile_read": (ctypes.c_int, [vp, ctypes.POINTER(ctypes.c_double),
                                           ctypes.POINTER(ctypes.c_double),
                                           ctypes.POINTER(ctypes.c_double),
                                           ctypes.POINTER(i32)]),
        "rt_device_info": (ctypes.c_int, [vp, ctypes.c_char_p, i32, ctypes.POINTER(i32),
                                          ctypes.POINTER(ctypes.c_int64)]),
        "rt_cube_init": (None, [vp]),
        "rt_cube_scale": (None, [vp, f32, f32, f32]),
        "rt_cube_rotate": (None, [vp, f32, f32, f32]),
        "rt_cube_translate": (None, [vp, f32, f32, f32]),
        "rt_deg_to_rad": (f32, [f32]),
        "rt_primary_ray_dir": (None, [vp]),
        "rt_scene_reference": (ctypes.c_int, [i32, ctypes.c_uint32, vp, vp, vp, vp, vp,
                                              ctypes.POINTER(i32), ctypes.POINTER(i32)]),
        "rt_scene_synthetic": (ctypes.c_int, [i32, i32, i32, i32, ctypes.c_uint64, f32, vp,
                                              vp, vp, vp, vp]),
        "rt_pack_rgba8": (None, [vp, ctypes.c_int64, vp]),
        "rt_abi_version": (ctypes.c_int, []),
        "rt_fnv1a64": (ctypes.c_uint64, [vp, ctypes.c_int64, ctypes.c_uint64]),
        "rt_selftest_fp32": (ctypes.c_int, [vp, vp, i32, vp, vp]),
        "rt_debug_triangle_box": (ctypes.c_int, [vp, vp, vp, vp, i32, i32, i32, vp, vp]),
        "rt_debug_sphere_box": (ctypes.c_int, [vp, f32, vp, i32, i32, i32, vp, vp]),
        "rt_debug_set_trace_mode": (ctypes.c_int, [vp, ctypes.c_int]),
        "rt_reserve": (ctypes.c_int, [vp, i32, i32, i32, i32, i32]),
        "rt_last_kernel": (ctypes.c_int, [vp, ctypes.POINTER(i32)]),
        "rt_debug_set_list_budget": (ctypes.c_int, [vp, ctypes.c_int64]),
        "rt_debug_set_bin_masks": (ctypes.c_int, [vp, ctypes.c_int]),
        "rt_debug_set_small_path": (ctypes.c_int, [vp, ctypes.c_int]),
        "rt_debug_set_coarse_cull": (ctypes.c_int, [vp, ctypes.c_int]),
        "rt_debug_set_tile_variant": (ctypes.c_int, [vp, ctypes.c_int]),
        "rt_debug_set_coarse_cull_tri": (ctypes.c_int, [vp, ctypes.c_int]),
        "rt_debug_set_coarse_cull_overdraw": (ctypes.c_int, [vp, ctypes.c_int]),
        "rt_debug_set_small_fused": (ctypes.c_int, [vp, ctypes.c_int]),
        "rt_debug_set_trace_split": (ctypes.c_int, [vp, ctypes.c_int]),
        "rt_debug_set_coarse_waves": (ctypes.c_int, [vp, ctypes.c_int]),
        "rt_debug_set_trace_bin": (ctypes.c_int, [vp, ctypes.c_int]),
        "rt_debug_set_verdict_copy": (ctypes.c_int, [vp, ctypes.c_int]),
        "rt_debug_last_overdraw": (ctypes.c_int, [vp, ctypes.POINTER(ctypes.c_double)]),
        "rt_debug_triangle_t_bounds": (ctypes.c_int, [vp, vp, vp, vp, i32, i32, i32, i32, i32,
                                                      i32, i32, vp]),
        "rt_debug_triangle_box_wide": (ctypes.c_int, [vp, vp, vp, vp, i32, i32, i32, vp, vp]),
        "rt_cube_build_device": (ctypes.c_int, [vp, vp, vp, i32, vp, vp, vp]),
        "rt_scene_synthetic_device": (ctypes.c_int, [vp, i32, i32, i32, i32, ctypes.c_uint64,
                                                     f32, vp, vp, vp, vp, vp, vp]),
        "rt_debug_glibc_sincosf": (ctypes.c_int, [vp, ctypes.c_int64, vp, vp]),
        "rt_selftest_sincosf": (ctypes.c_int, [vp, vp, ctypes.c_int64, vp, vp]),
    }
    for name, (res, args) in sig.items():
        if name in DIAG_SYMBOLS and not hasattr(lib, name):
            continue  # the default (non-diagnostics) build
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _LIB = lib
    return lib


def _error_string(status: int) -> str:
    try:
        return library().rt_error_string(status).decode()
    except Exception:  # pragma: no cover - library missing while formatting
        return "unknown"


def _ptr(a: Optional[np.ndarray]) -> Optional[int]:
    return None if a is None else a.ctypes.data


def _check(status: int, what: str) -> None:
    if status != RT_OK:
        raise RtError(status, what)


# ---------------------------------------------------------------------------
# host-side scene helpers (Cube.cpp, Utility.cpp, MainState.cpp:37-39)
# ---------------------------------------------------------------------------
def deg_to_rad(deg: float) -> float:
    return float(library().rt_deg_to_rad(deg))


def primary_ray_dir() -> np.ndarray:
    out = np.zeros(4, np.float32)
    library().rt_primary_ray_dir(_ptr(out))
    return out


def cube_packed(ops) -> np.ndarray:
    """Unit cube transformed by ops [("scale"|"rotate"|"translate", x, y, z), ...]."""
    lib = library()
    v = np.zeros((36, 4), np.float32)
    lib.rt_cube_init(_ptr(v))
    fns = {"scale": lib.rt_cube_scale, "rotate": lib.rt_cube_rotate,
           "translate": lib.rt_cube_translate}
    for op, x, y, z in ops:
        fns[op](_ptr(v), x, y, z)
    return v


# rt_cube_op (include/rt_hip.h): one Cube method call; rotate angles in radians
CUBE_OP_DTYPE = np.dtype([("op", "<i4"), ("x", "<f4"), ("y", "<f4"), ("z", "<f4")])
CUBE_OPS = {"scale": 1, "rotate": 2, "translate": 3}


def cube_ops(programs) -> Tuple[np.ndarray, np.ndarray]:
    """Pack per-cube op lists [[("scale"|"rotate"|"translate", x, y, z), ...], ...]
    into the (rt_cube_op array, int32 offsets) pair rt_cube_build_device reads."""
    flat = [(CUBE_OPS[op], x, y, z) for prog in programs for op, x, y, z in prog]
    ops = np.array(flat, CUBE_OP_DTYPE) if flat else np.zeros(0, CUBE_OP_DTYPE)
    offsets = np.zeros(len(programs) + 1, np.int32)
    offsets[1:] = np.cumsum([len(p) for p in programs])
    return ops, offsets


def debug_glibc_sincosf(x: np.ndarray) -> Tuple[np.ndarray, np.ndarray]:
    """Host run of the device's restatement of glibc sinf / cosf."""
    x = np.ascontiguousarray(x, np.float32).reshape(-1)
    s, c = np.empty_like(x), np.empty_like(x)
    _check(library().rt_debug_glibc_sincosf(_ptr(x), x.size, _ptr(s), _ptr(c)),
           "rt_debug_glibc_sincosf")
    return s, c


def pack_rgba8(frame: np.ndarray) -> np.ndarray:
    """Texture conversion (MainState.cpp:1023-1037) of an int32x4 frame."""
    frame = np.ascontiguousarray(frame, dtype=np.int32)
    n = frame.size // 4
    out = np.zeros(frame.shape[:-1], np.uint32)
    library().rt_pack_rgba8(_ptr(frame), n, _ptr(out))
    return out


FNV1A64_BASIS = 0xcbf29ce484222325


def fnv1a64(words, basis: int = FNV1A64_BASIS) -> int:
    """FNV-1a-64 over a frame's 32-bit words in memory order (rt_fnv1a64):
    the known-answer checksum of the committed fixtures.  `words`: a numpy
    array (any 4-byte dtype, C-contiguous) or a CPU torch tensor."""
    if not isinstance(words, np.ndarray):
        words = words.contiguous().numpy()
    words = np.ascontiguousarray(words)
    if words.dtype.itemsize != 4:
        raise ValueError(f"fnv1a64 hashes 32-bit words, got {words.dtype}")
    return int(library().rt_fnv1a64(_ptr(words), words.size, basis))


@dataclass
class Scene:
    """The reference's scene vectors (MainState.h:99-106), cubes flattened
    to 36 world-space float4 vertices each (MainState.cpp:646-655)."""

    sphere_origins: np.ndarray = field(default_factory=lambda: np.zeros((0, 4), np.float32))
    sphere_radius: np.ndarray = field(default_factory=lambda: np.zeros((0,), np.float32))
    sphere_colours: np.ndarray = field(default_factory=lambda: np.zeros((0, 4), np.float32))
    cube_vertices: np.ndarray = field(default_factory=lambda: np.zeros((0, 36, 4), np.float32))
    cube_colours: np.ndarray = field(default_factory=lambda: np.zeros((0, 4), np.float32))
    lights: np.ndarray = field(default_factory=lambda: np.zeros((0, 4), np.float32))

    def __post_init__(self):
        self.sphere_origins = np.ascontiguousarray(self.sphere_origins, np.float32).reshape(-1, 4)
        self.sphere_radius = np.ascontiguousarray(self.sphere_radius, np.float32).reshape(-1)
        self.sphere_colours = np.ascontiguousarray(self.sphere_colours, np.float32).reshape(-1, 4)
        self.cube_vertices = np.ascontiguousarray(self.cube_vertices, np.float32).reshape(-1, 36, 4)
        self.cube_colours = np.ascontiguousarray(self.cube_colours, np.float32).reshape(-1, 4)
        self.lights = np.ascontiguousarray(self.lights, np.float32).reshape(-1, 4)
        if not (len(self.sphere_origins) == len(self.sphere_radius) == len(self.sphere_colours)):
            raise ValueError("sphere arrays disagree in length")
        if len(self.cube_vertices) != len(self.cube_colours):
            raise ValueError("cube arrays disagree in length")

    @property
    def num_spheres(self) -> int:
        return len(self.sphere_radius)

    @property
    def num_cubes(self) -> int:
        return len(self.cube_colours)

    def as_c(self) -> _Scene:
        return _Scene(_ptr(self.sphere_origins), _ptr(self.sphere_radius),
                      _ptr(self.sphere_colours), self.num_spheres, _ptr(self.cube_vertices),
                      _ptr(self.cube_colours), self.num_cubes, _ptr(self.lights),
                      len(self.lights))

    @classmethod
    def reference(cls, scene_id: int, seed: int = 1) -> "Scene":
        """MainState::createScene1/2/3 (MainState.cpp:419-639) after
        Random::init(seed)."""
        so = np.zeros((100, 4), np.float32)
        sr = np.zeros(100, np.float32)
        sc = np.zeros((100, 4), np.float32)
        cv = np.zeros((100, 36, 4), np.float32)
        cc = np.zeros((100, 4), np.float32)
        ns, nc = ctypes.c_int32(), ctypes.c_int32()
        _check(library().rt_scene_reference(scene_id, seed, _ptr(so), _ptr(sr), _ptr(sc),
                                            _ptr(cv), _ptr(cc), ctypes.byref(ns),
                                            ctypes.byref(nc)), "rt_scene_reference")
        return cls(so[:ns.value], sr[:ns.value], sc[:ns.value], cv[:nc.value], cc[:nc.value])

    @classmethod
    def synthetic(cls, width: int, height: int, n_spheres: int, n_cubes: int,
                  seed: int = 7, k: float = 1.0, n_lights: int = 0) -> "Scene":
        """SURVEY.md §8d synthetic N-sphere/M-cube scene; lights are carried
        (the reference has no lighting model, so they never change pixels)."""
        so = np.zeros((n_spheres, 4), np.float32)
        sr = np.zeros(n_spheres, np.float32)
        sc = np.zeros((n_spheres, 4), np.float32)
        cv = np.zeros((n_cubes, 36, 4), np.float32)
        cc = np.zeros((n_cubes, 4), np.float32)
        _check(library().rt_scene_synthetic(width, height, n_spheres, n_cubes, seed, k,
                                            _ptr(so), _ptr(sr), _ptr(sc), _ptr(cv), _ptr(cc)),
               "rt_scene_synthetic")
        lights = np.tile(np.array([[width / 2, height / 2, 200.0, 1.0]], np.float32),
                         (n_lights, 1))
        return cls(so, sr, sc, cv, cc, lights)


@dataclass
class Timing:
    total_us: float
    upload_us: float
    kernel_us: float
    download_us: float
    path: str


def render_multi(tracers, scene: Scene, width: int, height: int,
                 rows: Optional[Tuple[int, int]] = None, ray_dir: Optional[np.ndarray] = None,
                 ray_origins: Optional[np.ndarray] = None,
                 fmt: str = "i32x4") -> Tuple[np.ndarray, list]:
    """rt_render_multi: one frame (or row range) split into contiguous row
    bands over `tracers` (one RayTracer per device), rendered concurrently
    into one host frame.  Returns (frame, per-band Timing list)."""
    rb, re = rows if rows is not None else (0, height)
    d = primary_ray_dir() if ray_dir is None else np.ascontiguousarray(ray_dir, np.float32)
    org = None if ray_origins is None else np.ascontiguousarray(ray_origins, np.float32)
    if org is not None and org.size != 4 * width * height:
        raise ValueError("ray_origins must hold width*height float4")
    shape = (re - rb, width, 4) if fmt == "i32x4" else (re - rb, width)
    out = np.empty(shape, np.int32 if fmt == "i32x4" else np.uint32)
    ctxs = (ctypes.c_void_p * len(tracers))(*[t.handle.value for t in tracers])
    times = (_Timing * len(tracers))()
    sc = scene.as_c()
    _check(library().rt_render_multi(ctxs, len(tracers), ctypes.byref(sc), _ptr(d), _ptr(org),
                                     width, height, rb, re, _FORMATS[fmt], _ptr(out), times),
           "rt_render_multi")
    names = {RT_PATH_BINNED: "binned", RT_PATH_GENERIC: "generic"}
    return out, [Timing(t.total_us, t.upload_us, t.kernel_us, t.download_us,
                        names.get(t.path, "idle")) for t in times]


def host_register(buf: np.ndarray) -> None:
    """rt_host_register: page-lock a host frame (e.g. the `pixels` array) so
    frame downloads into it are direct DMA."""
    _check(library().rt_host_register(_ptr(buf), buf.nbytes), "rt_host_register")


def host_unregister(buf: np.ndarray) -> None:
    _check(library().rt_host_unregister(_ptr(buf)), "rt_host_unregister")


class RayTracer:
    """One HIP device context (rt_init / rt_destroy)."""

    def __init__(self, device: int = 0):
        lib = library()
        self._ctx = ctypes.c_void_p()
        _check(lib.rt_init(device, ctypes.byref(self._ctx)), "rt_init")
        self.device = device

    def close(self) -> None:
        if self._ctx:
            library().rt_destroy(self._ctx)
            self._ctx = ctypes.c_void_p()

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):  # pragma: no cover - interpreter teardown order
        try:
            self.close()
        except Exception:
            pass

    @property
    def handle(self) -> ctypes.c_void_p:
        return self._ctx

    def render(self, scene: Scene, width: int, height: int, rows: Optional[Tuple[int, int]] = None,
               ray_dir: Optional[np.ndarray] = None, ray_origins: Optional[np.ndarray] = None,
               fmt: str = "i32x4", path: str = "auto",
               out: Optional[np.ndarray] = None) -> Tuple[np.ndarray, Timing]:
        """Synchronous host-buffer render (rt_render_path).  Returns the frame
        (rows x width x 4 int32, or rows x width uint32 for rgba8), written
        into `out` when given (a reused buffer, like the reference's
        `pixels` vector, MainState.cpp:215, avoids first-touch page faults
        in the readback)."""
        rb, re = rows if rows is not None else (0, height)
        d = primary_ray_dir() if ray_dir is None else np.ascontiguousarray(ray_dir, np.float32)
        org = None if ray_origins is None else np.ascontiguousarray(ray_origins, np.float32)
        if org is not None and org.size != 4 * width * height:
            raise ValueError("ray_origins must hold width*height float4")
        shape = (re - rb, width, 4) if fmt == "i32x4" else (re - rb, width)
        dtype = np.int32 if fmt == "i32x4" else np.uint32
        if out is None:
            out = np.empty(shape, dtype)
        elif out.shape != shape or out.dtype != dtype or not out.flags.c_contiguous:
            raise ValueError(f"out must be a C-contiguous {dtype.__name__} array of {shape}")
        t = _Timing()
        sc = scene.as_c()
        _check(library().rt_render_path(self._ctx, ctypes.byref(sc), _ptr(d), _ptr(org), width,
                                        height, rb, re, _FORMATS[fmt], _PATHS[path], _ptr(out),
                                        ctypes.byref(t)), "rt_render")
        used = {RT_PATH_BINNED: "binned", RT_PATH_GENERIC: "generic"}.get(t.path, "?")
        return out, Timing(t.total_us, t.upload_us, t.kernel_us, t.download_us, used)

    def render_device(self, device_scene: dict, width: int, height: int, rows: Tuple[int, int],
                      out_ptr: int, ray_dir: Optional[np.ndarray] = None, fmt: str = "i32x4",
                      path: str = "auto", stream: int = 0, origins_ptr: int = 0) -> None:
        """Asynchronous device-pointer render (rt_render_device).  `device_scene`
        maps the rt_scene fields to device addresses (e.g. torch data_ptr())."""
        d = primary_ray_dir() if ray_dir is None else np.ascontiguousarray(ray_dir, np.float32)
        sc = _Scene(device_scene.get("sphere_origins"), device_scene.get("sphere_radius"),
                    device_scene.get("sphere_colours"), int(device_scene.get("num_spheres", 0)),
                    device_scene.get("cube_vertices"), device_scene.get("cube_colours"),
                    int(device_scene.get("num_cubes", 0)), None, 0)
        _check(library().rt_render_device(self._ctx, ctypes.byref(sc), _ptr(d),
                                          origins_ptr or None, width, height, rows[0], rows[1],
                                          _FORMATS[fmt], _PATHS[path], out_ptr, stream or None),
               "rt_render_device")

    def bind_render_device(self, device_scene: dict, width: int, height: int,
                           rows: Tuple[int, int], out_ptr: int,
                           ray_dir: Optional[np.ndarray] = None, fmt: str = "i32x4",
                           path: str = "auto", stream: int = 0, origins_ptr: int = 0):
        """render_device with its ctypes arguments built once: returns a
        zero-argument callable that enqueues the render (for per-frame loops
        over an unchanged device scene / frame buffer)."""
        d = primary_ray_dir() if ray_dir is None else np.ascontiguousarray(ray_dir, np.float32)
        sc = _Scene(device_scene.get("sphere_origins"), device_scene.get("sphere_radius"),
                    device_scene.get("sphere_colours"), int(device_scene.get("num_spheres", 0)),
                    device_scene.get("cube_vertices"), device_scene.get("cube_colours"),
                    int(device_scene.get("num_cubes", 0)), None, 0)
        fn = library().rt_render_device
        args = (self._ctx, ctypes.byref(sc), _ptr(d), ctypes.c_void_p(origins_ptr or None),
                width, height, rows[0], rows[1], _FORMATS[fmt], _PATHS[path],
                ctypes.c_void_p(out_ptr), ctypes.c_void_p(stream or None))
        keep = (d, sc)  # referenced by the ctypes pointers above

        def render() -> None:
            rc = fn(*args)
            if rc != RT_OK:
                _check(rc, "rt_render_device")
        render._keep = keep  # type: ignore[attr-defined]
        return render

    def shared_alloc(self, nbytes: int) -> Tuple[int, bytes]:
        """rt_shared_alloc: a device buffer on this context's GPU plus the
        64-byte IPC handle other ranks map it with.  Returns (ptr, handle)."""
        p, h = ctypes.c_void_p(), _IpcHandle()
        _check(library().rt_shared_alloc(self._ctx, nbytes, ctypes.byref(p), ctypes.byref(h)),
               "rt_shared_alloc")
        return p.value, bytes(h.bytes)

    def shared_open(self, handle: bytes) -> int:
        """rt_shared_open: map another process's rt_shared_alloc buffer into
        this context's device (peer access over xGMI)."""
        if len(handle) != 64:
            raise ValueError("an IPC handle is 64 bytes")
        h = _IpcHandle()
        ctypes.memmove(h.bytes, handle, 64)
        p = ctypes.c_void_p()
        _check(library().rt_shared_open(self._ctx, ctypes.byref(h), ctypes.byref(p)),
               "rt_shared_open")
        return p.value

    def shared_close(self, ptr: int) -> None:
        _check(library().rt_shared_close(self._ctx, ptr), "rt_shared_close")

    def shared_free(self, ptr: int) -> None:
        _check(library().rt_shared_free(self._ctx, ptr), "rt_shared_free")

    def profile(self, enable: bool) -> None:
        _check(library().rt_profile_enable(self._ctx, int(enable)), "rt_profile_enable")

    def profile_read(self) -> dict:
        a, b, c = ctypes.c_double(), ctypes.c_double(), ctypes.c_double()
        n = ctypes.c_int32()
        _check(library().rt_profile_read(self._ctx, ctypes.byref(a), ctypes.byref(b),
                                         ctypes.byref(c), ctypes.byref(n)), "rt_profile_read")
        return {"prep_ms": a.value, "bin_ms": b.value, "trace_ms": c.value, "renders": n.value}

    def set_trace_mode(self, mode: int) -> None:
        """Diagnostics ablation of the trace kernel (0 = normal).  Modes other
        than 0 need the diagnostics build (make RT_DIAG=1); the default
        library has only the real kernel."""
        lib = library()
        if not hasattr(lib, "rt_debug_set_trace_mode"):
            if mode:
                raise RtError(RT_ERR_UNSUPPORTED, "rt_debug_set_trace_mode (needs RT_DIAG=1)")
            return
        _check(lib.rt_debug_set_trace_mode(self._ctx, mode), "rt_debug_set_trace_mode")

    def reserve(self, width: int, rows: int, n_spheres: int, n_cubes: int,
                fmt: str = "i32x4") -> None:
        """rt_reserve: size the workspace for frames of this shape ahead of
        the first render (openCLInit's one-time setup, MainState.cpp:1290-1320)."""
        _check(library().rt_reserve(self._ctx, width, rows, n_spheres, n_cubes, _FORMATS[fmt]),
               "rt_reserve")

    def last_kernel(self) -> Optional[str]:
        """rt_last_kernel: the kernel the last render did its per-pixel work
        with ("trace3_kernel", "trace3_split_kernel" -- the default on small
        binned frames --, "trace_bin_kernel" -- binned frames without the
        coarse kernel --, "trace_small_kernel", "frame_small_kernel",
        "generic_kernel"; None before any render)."""
        k = ctypes.c_int32()
        _check(library().rt_last_kernel(self._ctx, ctypes.byref(k)), "rt_last_kernel")
        return KERNEL_NAMES.get(k.value)

    def set_list_budget(self, nbytes: int) -> None:
        """Diagnostics: coarse-list byte budget (0 = default); frames over it
        render as internal row bands."""
        _check(library().rt_debug_set_list_budget(self._ctx, nbytes), "rt_debug_set_list_budget")

    def set_small_path(self, enable: bool) -> None:
        """Scenes of at most 512 primitives: trace_small_kernel (default) or the
        general prep -> coarse -> trace path (diagnostics / tests)."""
        _check(library().rt_debug_set_small_path(self._ctx, int(enable)),
               "rt_debug_set_small_path")

    def set_small_fused(self, mode: int) -> None:
        """Scenes of at most 128 primitives: the one-kernel frame_small_kernel
        where its grid is resident at once (1, default), on every frame size
        (2), or prep + trace_small_kernel (0) (diagnostics / tests)."""
        _check(library().rt_debug_set_small_fused(self._ctx, int(mode)),
               "rt_debug_set_small_fused")

    def set_trace_split(self, waves: int) -> None:
        """Waves per wave tile in the binned trace: 0 = by frame size
        (trace3_split_kernel on small frames, default), 1 = trace3_kernel,
        2 / 4 = trace3_split_kernel with that many (diagnostics / tests)."""
        _check(library().rt_debug_set_trace_split(self._ctx, int(waves)),
               "rt_debug_set_trace_split")

    def set_coarse_waves(self, waves: int) -> None:
        """Waves per coarse bin: 0 = by band size (default), 1 / 2 / 4 / 8
        (diagnostics / tests)."""
        _check(library().rt_debug_set_coarse_waves(self._ctx, int(waves)),
               "rt_debug_set_coarse_waves")

    def set_trace_bin(self, mode: int) -> None:
        """Binned frames without the coarse kernel (trace_bin_kernel: every
        wave tile classifies its bin's candidates itself): 0 = automatic
        (default), 1 = wherever it applies, 2 = never (diagnostics / tests)."""
        _check(library().rt_debug_set_trace_bin(self._ctx, int(mode)),
               "rt_debug_set_trace_bin")

    def set_verdict_copy(self, copy: bool) -> None:
        """How the overdraw verdict reaches the host (rt_debug_set_verdict_copy):
        False (default) = the kernels store it into the mapped host word,
        True = a copy every 8th binned launch (the fallback; tests)."""
        _check(library().rt_debug_set_verdict_copy(self._ctx, int(bool(copy))),
               "rt_debug_set_verdict_copy")

    def last_overdraw(self) -> float:
        """rt_debug_last_overdraw: the last binned render's box overdraw, in
        frames (synchronises the device)."""
        v = ctypes.c_double()
        _check(library().rt_debug_last_overdraw(self._ctx, ctypes.byref(v)),
               "rt_debug_last_overdraw")
        return v.value

    def set_coarse_cull_tri(self, min_candidates: int) -> None:
        """Diagnostics: triangles join the coarse depth cull in bins with at
        least this many candidates (0 = never, negative = default)."""
        _check(library().rt_debug_set_coarse_cull_tri(self._ctx, int(min_candidates)),
               "rt_debug_set_coarse_cull_tri")

    def set_coarse_cull_overdraw(self, frames: int) -> None:
        """Diagnostics: ... and only in frames whose boxes cover the frame at
        least this many times (0 = every frame, negative = default)."""
        _check(library().rt_debug_set_coarse_cull_overdraw(self._ctx, int(frames)),
               "rt_debug_set_coarse_cull_overdraw")

    def set_tile_variant(self, variant: int) -> None:
        """Diagnostics: the binned path's wave-tile build (0 = by frame size,
        1 = 16x16, 2 = the wide 128x2 tiles)."""
        _check(library().rt_debug_set_tile_variant(self._ctx, int(variant)),
               "rt_debug_set_tile_variant")

    def set_coarse_cull(self, min_candidates) -> None:
        """Diagnostics: the coarse kernel's depth cull of sphere candidates,
        in bins with at least `min_candidates` candidates (True = every bin,
        False / 0 = off: every candidate the tile classifier keeps stays)."""
        _check(library().rt_debug_set_coarse_cull(self._ctx, int(min_candidates)),
               "rt_debug_set_coarse_cull")

    def set_bin_masks(self, enable: bool) -> None:
        """Diagnostics: coarse binning from the separable bin masks (default)
        or from a scan of every primitive's box."""
        _check(library().rt_debug_set_bin_masks(self._ctx, int(bool(enable))),
               "rt_debug_set_bin_masks")

    def device_info(self) -> dict:
        name = ctypes.create_string_buffer(256)
        cu, mem = ctypes.c_int32(), ctypes.c_int64()
        _check(library().rt_device_info(self._ctx, name, 256, ctypes.byref(cu),
                                        ctypes.byref(mem)), "rt_device_info")
        return {"name": name.value.decode(), "cus": cu.value, "total_mem": mem.value}

    def cube_build_device(self, ops_ptr: int, offsets_ptr: int, n_cubes: int,
                          vertices_out_ptr: int, vertices_in_ptr: int = 0,
                          stream: int = 0) -> None:
        """rt_cube_build_device: cubes from the unit cube (or vertices_in) through
        their rt_cube_op programs, on the device.  All device pointers."""
        _check(library().rt_cube_build_device(self._ctx, ops_ptr or None, offsets_ptr or None,
                                              n_cubes, vertices_in_ptr or None,
                                              vertices_out_ptr or None, stream or None),
               "rt_cube_build_device")

    def scene_synthetic_device(self, width: int, height: int, n_spheres: int, n_cubes: int,
                               seed: int, k: float, device_scene: dict, stream: int = 0) -> None:
        """rt_scene_synthetic_device into the device arrays of `device_scene`
        (rt_scene field name -> device address)."""
        g = device_scene.get
        _check(library().rt_scene_synthetic_device(
            self._ctx, width, height, n_spheres, n_cubes, seed, k, g("sphere_origins"),
            g("sphere_radius"), g("sphere_colours"), g("cube_vertices"), g("cube_colours"),
            stream or None), "rt_scene_synthetic_device")

    def selftest_sincosf(self, x_ptr: int, n: int, sin_ptr: int, cos_ptr: int) -> None:
        """The device's glibc sinf / cosf restatement on n device floats."""
        _check(library().rt_selftest_sincosf(self._ctx, x_ptr, n, sin_ptr, cos_ptr),
               "rt_selftest_sincosf")

    def selftest_fp32(self, x: np.ndarray) -> Tuple[np.ndarray, np.ndarray]:
        x = np.ascontiguousarray(x, np.float32)
        s, q = np.empty_like(x), np.empty_like(x)
        _check(library().rt_selftest_fp32(self._ctx, _ptr(x), x.size, _ptr(s), _ptr(q)),
               "rt_selftest_fp32")
        return s, q


def debug_triangle_prep(v0, v1, v2, ray_dir, width, row_begin, row_end):
    """Host evaluation of the prep kernel's triangle box and tile classifier
    (the same __host__ __device__ code).  Returns (valid, box[4], cls[8])."""
    a = [np.ascontiguousarray(v, np.float32)[:3].copy() for v in (v0, v1, v2)]
    d = np.ascontiguousarray(ray_dir, np.float32)
    box = np.zeros(4, np.int32)
    cls = np.zeros(8, np.float32)
    ok = library().rt_debug_triangle_box(_ptr(a[0]), _ptr(a[1]), _ptr(a[2]), _ptr(d), width,
                                         row_begin, row_end, _ptr(box), _ptr(cls))
    return bool(ok), box, cls


def debug_triangle_prep_wide(v0, v1, v2, ray_dir, width, row_begin, row_end):
    """debug_triangle_prep of the wide-tile (128x2) build (its classifier margin
    covers 128-pixel tile spans: kTileSpan = max(kWaveTile, kWaveTileH))."""
    a = [np.ascontiguousarray(v, np.float32)[:3].copy() for v in (v0, v1, v2)]
    d = np.ascontiguousarray(ray_dir, np.float32)
    box = np.zeros(4, np.int32)
    cls = np.zeros(8, np.float32)
    ok = library().rt_debug_triangle_box_wide(_ptr(a[0]), _ptr(a[1]), _ptr(a[2]), _ptr(d), width,
                                              row_begin, row_end, _ptr(box), _ptr(cls))
    return bool(ok), box, cls


def debug_triangle_t_bounds(v0, v1, v2, ray_dir, width, row_begin, row_end, xa, xb, ya, yb):
    """Host evaluation of the coarse kernel's fp64 bounds of the trace's
    computed t over pixels [xa, xb] x [ya, yb] (None without a bound)."""
    a = [np.ascontiguousarray(v, np.float32)[:3].copy() for v in (v0, v1, v2)]
    d = np.ascontiguousarray(ray_dir, np.float32)
    out = np.zeros(2, np.float64)
    ok = library().rt_debug_triangle_t_bounds(_ptr(a[0]), _ptr(a[1]), _ptr(a[2]), _ptr(d), width,
                                              row_begin, row_end, xa, xb, ya, yb, _ptr(out))
    return (float(out[0]), float(out[1])) if ok else None


def debug_sphere_prep(origin, radius, ray_dir, width, row_begin, row_end):
    """Host evaluation of the prep kernel's sphere box and classifier."""
    o = np.ascontiguousarray(origin, np.float32)
    d = np.ascontiguousarray(ray_dir, np.float32)
    box = np.zeros(4, np.int32)
    cls = np.zeros(8, np.float32)
    ok = library().rt_debug_sphere_box(_ptr(o), float(radius), _ptr(d), width, row_begin,
                                       row_end, _ptr(box), _ptr(cls))
    return bool(ok), box, cls


def encode_png(filename: str, rgba8: np.ndarray) -> None:
    """Write an RGBA8 frame (uint32 H x W from pack_rgba8, or uint8 H x W x 4)
    as an 8-bit RGBA PNG, the format lodepng::encode writes for the reference
    (MainState.cpp:410-417).  Plain zlib, filter type 0 on every scanline."""
    import struct
    import zlib

    px = np.ascontiguousarray(rgba8)
    if px.dtype != np.uint8:
        px = px.astype("<u4").view(np.uint8).reshape(px.shape[0], px.shape[1], 4)
    h, w = px.shape[:2]
    raw = np.zeros((h, 1 + 4 * w), np.uint8)
    raw[:, 1:] = px.reshape(h, 4 * w)

    def chunk(kind: bytes, data: bytes) -> bytes:
        return (struct.pack(">I", len(data)) + kind + data +
                struct.pack(">I", zlib.crc32(kind + data) & 0xFFFFFFFF))

    png = (b"\x89PNG\r\n\x1a\n" +
           chunk(b"IHDR", struct.pack(">IIBBBBB", w, h, 8, 6, 0, 0, 0)) +
           chunk(b"IDAT", zlib.compress(raw.tobytes(), 6)) + chunk(b"IEND", b""))
    with open(filename, "wb") as f:
        f.write(png)


class MainState:
    """Headless mirror of the reference's MainState trace flow
    (MainState.cpp:135-239 update, :419-639 scenes, :641 executeRayTracerOpenCL).

    ``execute_ray_tracer()`` leaves the int32x4 frame in ``pixels`` (a flat
    int32 array of 4*W*H, as the reference's std::vector<int>) and the wall
    time in ``time_taken`` (µs, the reference's timer scope :662-894)."""

    def __init__(self, width: int = 640, height: int = 480, device: int = 0):
        self.width, self.height = width, height
        self.pixel_count = width * height  # :34
        self.ray_dir = primary_ray_dir()   # :37-39
        self.current_scene = 1
        self.scene = Scene()
        self.pixels = np.zeros(0, np.int32)
        self.time_taken = 0.0
        self._rt = RayTracer(device)       # openCLInit, :52

    def create_scene(self, scene_id: int, seed: int = 1) -> None:
        self.current_scene = scene_id
        self.scene = Scene.reference(scene_id, seed)

    def createScene1(self, seed: int = 1):  # noqa: N802 - reference names
        self.create_scene(1, seed)

    def createScene2(self, seed: int = 1):  # noqa: N802
        self.create_scene(2, seed)

    def createScene3(self, seed: int = 1):  # noqa: N802
        self.create_scene(3, seed)

    def execute_ray_tracer(self) -> np.ndarray:
        frame, t = self._rt.render(self.scene, self.width, self.height, ray_dir=self.ray_dir)
        self.pixels = frame.reshape(-1)
        self.time_taken = t.total_us
        return frame

    executeRayTracerOpenCL = execute_ray_tracer  # noqa: N815 - the replaced entry

    def generate_image_from_pixels(self) -> np.ndarray:
        """RGBA8 Texture content (MainState.cpp:974-1045)."""
        return pack_rgba8(self.pixels.reshape(self.height, self.width, 4))

    def encode_png(self, filename: str) -> None:
        """MainState::encodePNG (MainState.cpp:410-417; the reference's call
        site at :971 is commented out): the current frame as an RGBA8 PNG."""
        encode_png(filename, self.generate_image_from_pixels())

    def close(self):
        self._rt.close()
