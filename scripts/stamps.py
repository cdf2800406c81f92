"""Read the per-phase s_memtime sums of an RT_STAMPS diagnostics build
(never quote its run time: the stamps serialise the phases)."""
import ctypes
import sys
from pathlib import Path

import numpy as np

REPO = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(REPO))


def main(path, mode=0, width=4096, height=4096, spheres=256, cubes=64, seed=3, reps=10):
    import torch  # noqa: F401  (one HIP runtime)
    import __graft_entry__
    pkg = __graft_entry__.load_package()
    lib = ctypes.CDLL(path, mode=ctypes.RTLD_LOCAL)
    ctx = ctypes.c_void_p()
    assert lib.rt_init(0, ctypes.byref(ctx)) == 0
    assert lib.rt_debug_set_trace_mode(ctx, mode) == 0
    scene = pkg.Scene.synthetic(width, height, spheres, cubes, seed=seed, k=width / 640)
    sc = scene.as_c()
    out = np.empty((height, width, 4), np.int32)
    buf = (ctypes.c_ulonglong * 16)()
    lib.rt_render_path.argtypes = [ctypes.c_void_p, ctypes.POINTER(pkg._Scene), ctypes.c_void_p,
                                   ctypes.c_void_p] + [ctypes.c_int32] * 6 + [ctypes.c_void_p,
                                                                             ctypes.c_void_p]
    d = pkg.primary_ray_dir()
    assert lib.rt_render_path(ctx, ctypes.byref(sc), d.ctypes.data, None, width, height, 0,
                              height, 0, 1, out.ctypes.data, None) == 0
    lib.rt_debug_read_stamps(ctx, buf)
    assert lib.rt_render_path(ctx, ctypes.byref(sc), d.ctypes.data, None, width, height, 0,
                              height, 0, 1, out.ctypes.data, None) == 0
    assert lib.rt_debug_read_stamps(ctx, buf) == 0  # one launch: per-wave slots
    v = list(buf)
    waves = v[5]
    names = ["stage+barrier", "filter", "walk", "shade", "store issue"]
    tot = sum(v[:5])
    print(f"mode {mode}: waves {waves}  per-wave cycles:")
    for i, n in enumerate(names):
        print(f"  {n:14s} {v[i] / waves:9.0f}  ({100 * v[i] / tot:4.1f}%)")
    print(f"  triangle candidates/wave {v[6] / waves:.2f} (tile-inside {v[7] / waves:.2f}), "
          f"sphere candidates/wave {v[8] / waves:.2f}")


if __name__ == "__main__":
    for m in (sys.argv[2:] or ["0"]):
        main(sys.argv[1], int(m))
