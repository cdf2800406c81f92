"""Runs the reference's own OpenCL kernel (rayTracer.cl, compiled unmodified
for gfx950 into oracle/_ref/rayTracer_gfx950.co by oracle/Makefile) on the
GPU through the HIP module API -- TEST INFRASTRUCTURE ONLY: it is the
reference side of a check (tests/test_reference_kernel.py), never a product
path.  The launch mirrors the reference's dispatch (MainState.cpp:841-869):
explicit ray origins (x, y, 0, 1) per pixel (MainState.cpp:44-50), one work
item per pixel; the kernel has no bounds check, so the buffers are padded to
whole workgroups."""
import ctypes
from pathlib import Path
from typing import Optional

import numpy as np

REPO = Path(__file__).resolve().parents[1]
CODE_OBJECT = REPO / "oracle" / "_ref" / "rayTracer_gfx950.co"


class _Float4(ctypes.Structure):
    _fields_ = [("x", ctypes.c_float), ("y", ctypes.c_float), ("z", ctypes.c_float),
                ("w", ctypes.c_float)]


class ReferenceKernel:
    BLOCK = 64

    def __init__(self, path: Path = CODE_OBJECT, device: int = 0):
        self.hip = ctypes.CDLL("libamdhip64.so")
        vp = ctypes.c_void_p
        self.hip.hipModuleLaunchKernel.argtypes = [vp] + [ctypes.c_uint] * 7 + [
            vp, ctypes.POINTER(vp), ctypes.POINTER(vp)]
        self.hip.hipMalloc.argtypes = [ctypes.POINTER(vp), ctypes.c_size_t]
        self.hip.hipMemcpy.argtypes = [vp, vp, ctypes.c_size_t, ctypes.c_int]
        self.hip.hipFree.argtypes = [vp]
        self.hip.hipModuleLoad.argtypes = [ctypes.POINTER(vp), ctypes.c_char_p]
        self.hip.hipModuleGetFunction.argtypes = [ctypes.POINTER(vp), vp, ctypes.c_char_p]
        self.hip.hipModuleUnload.argtypes = [vp]
        self.hip.hipEventCreate.argtypes = [ctypes.POINTER(vp)]
        self.hip.hipEventRecord.argtypes = [vp, vp]
        self.hip.hipEventSynchronize.argtypes = [vp]
        self.hip.hipEventDestroy.argtypes = [vp]
        self.hip.hipEventElapsedTime.argtypes = [ctypes.POINTER(ctypes.c_float), vp, vp]
        self._check(self.hip.hipSetDevice(device), "hipSetDevice")
        self.module = vp()
        self._check(self.hip.hipModuleLoad(ctypes.byref(self.module), str(path).encode()),
                    "hipModuleLoad")
        self.fn = vp()
        self._check(self.hip.hipModuleGetFunction(ctypes.byref(self.fn), self.module,
                                                  b"rayTracer"), "hipModuleGetFunction")

    @staticmethod
    def _check(rc: int, what: str):
        if rc != 0:
            raise RuntimeError(f"{what} failed: hipError {rc}")

    def _upload(self, a: np.ndarray, allocs: list) -> ctypes.c_void_p:
        a = np.ascontiguousarray(a)
        p = ctypes.c_void_p()
        self._check(self.hip.hipMalloc(ctypes.byref(p), max(a.nbytes, 256)), "hipMalloc")
        allocs.append(p)
        if a.nbytes:
            self._check(self.hip.hipMemcpy(p, a.ctypes.data, a.nbytes, 1), "hipMemcpy H2D")
        return p

    def trace(self, scene, width: int, height: int, ray_dir: np.ndarray,
              ray_origins: Optional[np.ndarray] = None, timed_reps: int = 0):
        """The frame (H, W, 4) int32; with timed_reps > 0 also the kernel's
        milliseconds per launch (HIP events around timed_reps launches on the
        null stream, after the first), buffers resident."""
        n_px = width * height
        grid = (n_px + self.BLOCK - 1) // self.BLOCK
        padded = grid * self.BLOCK
        org = np.zeros((padded, 4), np.float32)
        if ray_origins is None:
            ys, xs = np.divmod(np.arange(n_px, dtype=np.int64), width)
            org[:n_px, 0], org[:n_px, 1], org[:n_px, 3] = xs, ys, 1.0
        else:
            org[:n_px] = np.asarray(ray_origins, np.float32).reshape(n_px, 4)
        so = np.ascontiguousarray(scene.sphere_origins, np.float32).reshape(-1, 4)
        sr = np.ascontiguousarray(scene.sphere_radius, np.float32).reshape(-1)
        sc = np.ascontiguousarray(scene.sphere_colours, np.float32).reshape(-1, 4)
        cv = np.ascontiguousarray(scene.cube_vertices, np.float32).reshape(-1, 36, 4)
        cc = np.ascontiguousarray(scene.cube_colours, np.float32).reshape(-1, 4)
        assert len(so) == len(sr) == len(sc) and len(cv) == len(cc)
        allocs: list = []
        try:
            out = self._upload(np.zeros((padded, 4), np.int32), allocs)
            d_so, d_sr, d_sc = (self._upload(a, allocs) for a in (so, sr, sc))
            d_cv, d_cc, d_org = (self._upload(a, allocs) for a in (cv, cc, org))
            d = np.asarray(ray_dir, np.float32)
            # kernel arguments, rayTracer.cl:111-114
            vals = [out, ctypes.c_int(len(sr)), d_so, d_sr, d_sc, ctypes.c_int(len(cc)), d_cv,
                    d_cc, d_org, _Float4(*(float(v) for v in d))]
            params = (ctypes.c_void_p * len(vals))(
                *(ctypes.cast(ctypes.pointer(v), ctypes.c_void_p) for v in vals))
            def launch():
                self._check(self.hip.hipModuleLaunchKernel(self.fn, grid, 1, 1, self.BLOCK, 1, 1,
                                                           0, None, params, None),
                            "hipModuleLaunchKernel")
            launch()
            self._check(self.hip.hipDeviceSynchronize(), "hipDeviceSynchronize")
            ms = None
            if timed_reps > 0:
                ev = [ctypes.c_void_p(), ctypes.c_void_p()]
                for e in ev:
                    self._check(self.hip.hipEventCreate(ctypes.byref(e)), "hipEventCreate")
                self._check(self.hip.hipEventRecord(ev[0], None), "hipEventRecord")
                for _ in range(timed_reps):
                    launch()
                self._check(self.hip.hipEventRecord(ev[1], None), "hipEventRecord")
                self._check(self.hip.hipEventSynchronize(ev[1]), "hipEventSynchronize")
                t = ctypes.c_float()
                self._check(self.hip.hipEventElapsedTime(ctypes.byref(t), ev[0], ev[1]),
                            "hipEventElapsedTime")
                for e in ev:
                    self.hip.hipEventDestroy(e)
                ms = t.value / timed_reps
            frame = np.zeros((padded, 4), np.int32)
            self._check(self.hip.hipMemcpy(frame.ctypes.data, out, frame.nbytes, 2),
                        "hipMemcpy D2H")
        finally:
            for p in allocs:
                self.hip.hipFree(p)
        frame = frame[:n_px].reshape(height, width, 4)
        return frame if timed_reps <= 0 else (frame, ms)

    def close(self):
        if self.module:
            self.hip.hipModuleUnload(self.module)
            self.module = ctypes.c_void_p()
