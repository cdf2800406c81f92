"""A/B timing of librt_hip.so variants in ONE process, interleaved rounds
(cdna_hip_programming.md §5.4 rule 24), on the bench's config-3 scene.
Every variant's frame is checked bit-exact against the first variant's.

    python scripts/bench_variants.py opencl-ray-tracer_amd/variants/librt_hip_*.so
"""
import argparse
import ctypes
import json
import statistics
import sys
import time
from pathlib import Path

import numpy as np

REPO = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(REPO))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("libs", nargs="+")
    ap.add_argument("--rounds", type=int, default=7)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--width", type=int, default=4096)
    ap.add_argument("--height", type=int, default=4096)
    ap.add_argument("--spheres", type=int, default=256)
    ap.add_argument("--cubes", type=int, default=64)
    ap.add_argument("--seed", type=int, default=3)
    ap.add_argument("--k", type=float, default=None)
    ap.add_argument("--ranks", type=int, default=1,
                    help="render rank 0's band of a frame and scene scaled for this many ranks "
                         "(bench.py's weak-scaling workload)")
    ap.add_argument("--format", default="i32x4", choices=("i32x4", "rgba8"))
    ap.add_argument("--scene", type=int, default=0,
                    help="reference scene 1-3 at 640x480 from tests/golden instead of a "
                         "synthetic scene")
    ap.add_argument("--kernels", action="store_true",
                    help="also per-kernel medians (rt_profile_*: HIP events on each kernel)")
    ap.add_argument("--modes", default="0",
                    help="comma list of trace-kernel ablation modes to time (0 = real)")
    args = ap.parse_args()
    import torch
    import __graft_entry__
    pkg = __graft_entry__.load_package()
    w, h = args.width, args.height
    k = args.k if args.k is not None else w / 640
    full_h = h * args.ranks
    if args.scene:
        with np.load(REPO / "tests" / "golden" / f"scene{args.scene}_640x480.npz") as z:
            scene = pkg.Scene(z["sphere_origins"], z["sphere_radius"], z["sphere_colours"],
                              z["cube_vertices"], z["cube_colours"])
        w, h, full_h = 640, 480, 480
    else:
        scene = pkg.Scene.synthetic(w, full_h, args.spheres * args.ranks,
                                    args.cubes * args.ranks, seed=args.seed, k=k)
    dev = torch.device("cuda:0")
    t = {n: torch.from_numpy(np.ascontiguousarray(getattr(scene, n))).to(dev)
         for n in ("sphere_origins", "sphere_radius", "sphere_colours", "cube_vertices",
                   "cube_colours")}
    sc = pkg._Scene(t["sphere_origins"].data_ptr(), t["sphere_radius"].data_ptr(),
                    t["sphere_colours"].data_ptr(), scene.num_spheres,
                    t["cube_vertices"].data_ptr(), t["cube_colours"].data_ptr(),
                    scene.num_cubes, None, 0)
    d = pkg.primary_ray_dir()
    stream = torch.cuda.Stream(dev)
    fmt = 0 if args.format == "i32x4" else 1
    out = torch.empty((h, w, 4) if fmt == 0 else (h, w), dtype=torch.int32, device=dev)
    libs = []
    for spec in args.libs:
        # "path@setter=value,...": the same library with rt_debug_set_<setter>
        # applied (e.g. @coarse_cull_tri=0), timed as a variant of its own
        path, _, sets = spec.partition("@")
        lib = ctypes.CDLL(path, mode=ctypes.RTLD_LOCAL)
        ctx = ctypes.c_void_p()
        assert lib.rt_init(0, ctypes.byref(ctx)) == 0
        for kv in filter(None, sets.split(",")):
            k, v = kv.split("=")
            fn = getattr(lib, f"rt_debug_set_{k}")
            fn.argtypes = [ctypes.c_void_p, ctypes.c_int64 if k == "list_budget" else ctypes.c_int]
            assert fn(ctx, int(v)) == 0, kv
        lib.rt_render_device.argtypes = [ctypes.c_void_p, ctypes.POINTER(pkg._Scene),
                                         ctypes.c_void_p, ctypes.c_void_p] + \
            [ctypes.c_int32] * 6 + [ctypes.c_void_p, ctypes.c_void_p]
        libs.append((Path(path).stem.replace("librt_hip_", "") + (f"@{sets}" if sets else ""),
                     lib, ctx))

    def run(lib, ctx, n):
        for _ in range(n):
            rc = lib.rt_render_device(ctx, ctypes.byref(sc), d.ctypes.data, None, w, full_h, 0,
                                      h, fmt, 0, out.data_ptr(), stream.cuda_stream)
            assert rc == 0

    ref = None
    for name, lib, ctx in libs:  # warmup + parity
        run(lib, ctx, 3)
        torch.cuda.synchronize()
        frame = out.cpu()
        if ref is None:
            ref = frame
        elif not torch.equal(frame, ref):
            print(f"PARITY MISMATCH {name}: {(frame != ref).any(-1).sum().item()} px", flush=True)
    modes = [int(m) for m in args.modes.split(",")]
    times = {f"{name}" + (f"/m{m}" if m else ""): [] for m in modes for name, _, _ in libs}
    for r in range(args.rounds):
        order = libs if r % 2 == 0 else libs[::-1]
        for m in modes:
            for name, lib, ctx in order:
                if m:  # ablations need the RT_DIAG=1 build (rt_hip_diag.h)
                    assert lib.rt_debug_set_trace_mode(ctx, m) == 0
                torch.cuda.synchronize()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(stream)
                run(lib, ctx, args.steps)
                e1.record(stream)
                torch.cuda.synchronize()
                if m:
                    lib.rt_debug_set_trace_mode(ctx, 0)
                times[f"{name}" + (f"/m{m}" if m else "")].append(
                    e0.elapsed_time(e1) / args.steps * 1e3)
    res = {n: {"median_us": round(statistics.median(v), 2), "min_us": round(min(v), 2)}
           for n, v in times.items()}
    if args.kernels:
        dbl = ctypes.c_double
        for name, lib, ctx in libs:
            ks = {"prep": [], "bin": [], "trace": []}
            for _ in range(args.rounds):
                lib.rt_profile_enable(ctx, 1)
                run(lib, ctx, args.steps)
                v = [dbl(), dbl(), dbl()]
                n = ctypes.c_int32()
                assert lib.rt_profile_read(ctx, *[ctypes.byref(x) for x in v], ctypes.byref(n)) == 0
                lib.rt_profile_enable(ctx, 0)
                for key, x in zip(ks, v):
                    ks[key].append(x.value * 1e3 / max(n.value, 1))
            res[name].update({f"{key}_us": round(statistics.median(x), 2) for key, x in ks.items()})
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
