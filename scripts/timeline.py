"""Per-wave timeline of one trace_kernel launch (RT_TIMELINE=1 build):
occupancy over time, phase durations, dispatch order.  Diagnostics only.

    python scripts/timeline.py opencl-ray-tracer_amd/variants/librt_hip_tl.so [mode] [fmt 0|1]
"""
import ctypes
import sys
from pathlib import Path

import numpy as np

REPO = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(REPO))


def main(path, mode=0, fmt=0, width=4096, height=4096, spheres=256, cubes=64, seed=3):
    import torch
    import __graft_entry__
    pkg = __graft_entry__.load_package()
    lib = ctypes.CDLL(path, mode=ctypes.RTLD_LOCAL)
    ctx = ctypes.c_void_p()
    assert lib.rt_init(0, ctypes.byref(ctx)) == 0
    scene = pkg.Scene.synthetic(width, height, spheres, cubes, seed=seed, k=width / 640)
    dev = torch.device("cuda:0")
    t = {n: torch.from_numpy(np.ascontiguousarray(getattr(scene, n))).to(dev)
         for n in ("sphere_origins", "sphere_radius", "sphere_colours", "cube_vertices",
                   "cube_colours")}
    sc = pkg._Scene(t["sphere_origins"].data_ptr(), t["sphere_radius"].data_ptr(),
                    t["sphere_colours"].data_ptr(), scene.num_spheres,
                    t["cube_vertices"].data_ptr(), t["cube_colours"].data_ptr(),
                    scene.num_cubes, None, 0)
    lib.rt_render_device.argtypes = [ctypes.c_void_p, ctypes.POINTER(pkg._Scene),
                                     ctypes.c_void_p, ctypes.c_void_p] + \
        [ctypes.c_int32] * 6 + [ctypes.c_void_p, ctypes.c_void_p]
    d = pkg.primary_ray_dir()
    out = torch.empty((height, width, 4) if fmt == 0 else (height, width), dtype=torch.int32,
                      device=dev)
    n_waves = width * height // 256  # 256-pixel wave tiles
    tl = torch.zeros((n_waves * 8,), dtype=torch.int32, device=dev)
    assert lib.rt_debug_set_timeline(ctx, ctypes.c_void_p(tl.data_ptr())) == 0
    assert lib.rt_debug_set_trace_mode(ctx, mode) == 0
    stream = torch.cuda.Stream(dev)
    for _ in range(5):
        assert lib.rt_render_device(ctx, ctypes.byref(sc), d.ctypes.data, None, width, height,
                                    0, height, fmt, 0, out.data_ptr(), stream.cuda_stream) == 0
    torch.cuda.synchronize()
    v = tl.cpu().numpy().view(np.uint32).reshape(n_waves, 8).astype(np.int64)
    t0 = v[:, 0] - v[:, 0].min()
    t1 = v[:, 1] - v[:, 0].min()
    t2 = v[:, 2] - v[:, 0].min()
    t3 = v[:, 3] - v[:, 0].min()
    cyc = (v[:, 5] - v[:, 4]) % (1 << 32)
    hwid, xcc = v[:, 6], v[:, 7] & 0xF
    span = t3.max()
    life = t3 - t0
    us = 0.01  # realtime tick = 10 ns
    print(f"kernel span (first entry -> last store issue): {span * us:.1f} us")
    print(f"clock estimate: {np.median(cyc / np.maximum(life, 1)) / 10:.2f} GHz (memtime/realtime)")

    def pct(a, name):
        q = np.percentile(a * us, [10, 50, 90, 99])
        print(f"{name:>22}: mean {a.mean() * us:6.2f}  p10 {q[0]:6.2f}  p50 {q[1]:6.2f}"
              f"  p90 {q[2]:6.2f}  p99 {q[3]:6.2f} us")
    pct(life, "wave life")
    pct(t1 - t0, "stage (+filter in t2)")
    pct(t2 - t1, "filter+walk")
    pct(t3 - t2, "shade+store issue")
    # occupancy: waves alive per SIMD over time
    edges = np.linspace(0, span, 21)
    print("time(us)  alive-waves/SIMD  started  finished  store-issue TB/s  mean walk of finished")
    tile_bytes = width * height * (16 if fmt == 0 else 4) // n_waves
    for a, b in zip(edges[:-1], edges[1:]):
        mid = (a + b) / 2
        alive = ((t0 <= mid) & (t3 > mid)).sum() / 1024
        started = ((t0 >= a) & (t0 < b)).sum()
        fin = (t3 >= a) & (t3 < b)
        ended = fin.sum()
        rate = ended * tile_bytes / ((b - a) * us * 1e-6) / 1e12
        walk = (t2 - t1)[fin].mean() * us if ended else 0.0
        print(f"{mid * us:7.1f}  {alive:8.2f}  {started:8d}  {ended:8d}  {rate:8.2f}  {walk:8.2f}")
    first = np.sort(t3)[:64]
    print(f"first store issue at {first[0] * us:.2f} us, 64th at {first[-1] * us:.2f} us; "
          f"first wave entry at {t0.min() * us:.2f} us")
    # dispatch order
    order = np.argsort(t0, kind="stable")
    wg = np.arange(n_waves) // 4
    inv = np.corrcoef(order, np.arange(n_waves))[0, 1]
    print(f"dispatch order vs wave index correlation: {inv:.3f}")
    for x in range(8):
        m = xcc == x
        if m.any():
            print(f"xcc {x}: waves {m.sum():6d}  first start {t0[m].min() * us:6.2f}"
                  f"  last end {t3[m].max() * us:6.2f}  mean life {life[m].mean() * us:5.2f}")
    # per-CU (se, cu) balance
    cu = (xcc << 8) | ((hwid >> 8) & 0xF) | (((hwid >> 13) & 0x7) << 4)
    ids, counts = np.unique(cu, return_counts=True)
    print(f"CUs seen: {len(ids)}  waves/CU min {counts.min()} max {counts.max()}")
    np.save(REPO / "gpurun_out" / f"timeline_m{mode}_f{fmt}.npy", v)


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 0,
         int(sys.argv[3]) if len(sys.argv) > 3 else 0)
