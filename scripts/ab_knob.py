"""Interleaved A/B of one librt_hip.so runtime knob, in ONE process, on the
BASELINE configs (cdna_hip_programming.md §5.4 rule 24: interleave rounds,
compare medians).  Each setting's frame must be bit-identical to the first.

    python scripts/ab_knob.py --knob coarse_cull --values 0,1 --configs c3,c5d,c5s,band8

Prints one JSON line per config: median wall us per frame per setting, and
the per-kernel medians (HIP events on the kernels' dispatch packets).
"""
import argparse
import json
import statistics
import sys
import time
from pathlib import Path

import numpy as np

REPO = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(REPO))

# name: (width, frame height, rendered rows, spheres, cubes, seed, k)
CONFIGS = {
    "c1": (512, 512, (0, 512), 4, 1, 1, 0.8),
    "c2": (1920, 1080, (0, 1080), 16, 4, 2, 3.0),
    # reference scene 2's size: 640x480, 8 spheres + 10 cubes
    "s2": (640, 480, (0, 480), 8, 10, 1, 1.0),
    # 1080p with 256 / 512 primitives (the small path's 4- and 8-chunk instances)
    "p256": (1920, 1080, (0, 1080), 64, 16, 2, 3.0),
    "p512": (1920, 1080, (0, 1080), 128, 32, 2, 3.0),
    # small scenes on large frames (the one-kernel path's prep per workgroup)
    "uhd64": (3840, 2160, (0, 2160), 16, 4, 2, 6.0),
    "c3s64": (4096, 4096, (0, 4096), 16, 4, 3, 6.4),
    "c4s64": (8192, 8192, (0, 8192), 16, 4, 4, 12.8),
    "c3s16": (4096, 4096, (0, 4096), 4, 1, 1, 6.4),
    "c3": (4096, 4096, (0, 4096), 256, 64, 3, 6.4),
    "c3s": (4096, 4096, (0, 4096), 256, 64, 3, 1.0),
    # config 3's scene with 2x / 4x / 8x the object size (box overdraw ~11 / ~45 / ~180)
    "c3k2": (4096, 4096, (0, 4096), 256, 64, 3, 12.8),
    "c3k4": (4096, 4096, (0, 4096), 256, 64, 3, 25.6),
    "c3k8": (4096, 4096, (0, 4096), 256, 64, 3, 51.2),
    # config 3's scene at 1.5x object size (overdraw ~6)
    "c3k15": (4096, 4096, (0, 4096), 256, 64, 3, 9.6),
    # ... and at 1/6.4 .. 0.7x (the RGBA8 no-coarse crossover)
    "c3r2": (4096, 4096, (0, 4096), 256, 64, 3, 2.0),
    "c3r3": (4096, 4096, (0, 4096), 256, 64, 3, 3.2),
    "c3r45": (4096, 4096, (0, 4096), 256, 64, 3, 4.5),
    "c3r8": (4096, 4096, (0, 4096), 256, 64, 3, 8.0),
    "c4": (8192, 8192, (0, 8192), 192, 64, 4, 12.8),
    "c5d": (16384, 16384, (0, 16384), 4096, 0, 5, 25.6),
    "c5s": (16384, 16384, (0, 16384), 4096, 0, 5, 1.0),
    # rank 0's band of bench.py's 8-rank weak-scaling workload
    "band8": (4096, 32768, (0, 4096), 2048, 512, 3, 6.4),
    # rank 0's bands of configs 4 and 5 (8 ranks)
    "c4band": (8192, 8192, (0, 1024), 192, 64, 4, 12.8),
    "c4half": (8192, 8192, (0, 4096), 192, 64, 4, 12.8),
    "c4q3": (8192, 8192, (0, 3072), 192, 64, 4, 12.8),
    "c5half": (16384, 16384, (0, 8192), 4096, 0, 5, 25.6),
    "c5band4": (16384, 16384, (0, 4096), 4096, 0, 5, 25.6),
    "c5dband": (16384, 16384, (0, 2048), 4096, 0, 5, 25.6),
    "c5sband": (16384, 16384, (0, 2048), 4096, 0, 5, 1.0),
    # scenes of 4x and 16x config 3's object count at the same density
    "c3x4": (4096, 4096, (0, 4096), 1024, 256, 3, 6.4),
    "c3x16": (4096, 4096, (0, 4096), 4096, 1024, 3, 6.4),
    "c3x64": (4096, 4096, (0, 4096), 16384, 4096, 3, 6.4),
}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--knob", default="coarse_cull",
                    help="a RayTracer setter without set_ (coarse_cull, trace_bin, trace_bin_cull, ...)")
    ap.add_argument("--values", default="0,1")
    ap.add_argument("--configs", default="c3,c5d,c5s,band8")
    ap.add_argument("--format", default="i32x4", choices=("i32x4", "rgba8"))
    ap.add_argument("--fixed", action="append", default=[],
                    help="knob=value held for every setting (repeatable)")
    ap.add_argument("--rounds", type=int, default=7)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--no-check", action="store_true",
                    help="settings that change the frame on purpose (trace_mode ablations)")
    args = ap.parse_args()
    import torch
    import __graft_entry__

    pkg = __graft_entry__.load_package()
    dev = torch.device("cuda:0")
    stream = torch.cuda.Stream(dev)
    rt = pkg.RayTracer(0)
    if args.knob == "trace_path":
        # 0 = prep -> coarse -> trace, 1 = trace_bin_kernel (round 5 also
        # measured 2 = trace_tile_kernel, profiles/r05/trace_tile.patch)
        def setter(v):
            rt.set_trace_bin({0: 2, 1: 1}[v])
    else:
        setter = getattr(rt, "set_" + args.knob)
    for kv in args.fixed:
        name, val = kv.split("=")
        getattr(rt, "set_" + name)(int(val))
    values = [int(v) for v in args.values.split(",")]
    for cname in args.configs.split(","):
        w, h, (rb, re), ns, nc, seed, k = CONFIGS[cname]
        scene = pkg.Scene.synthetic(w, h, ns, nc, seed=seed, k=k)
        t = {n: torch.from_numpy(np.ascontiguousarray(getattr(scene, n))).to(dev)
             for n in ("sphere_origins", "sphere_radius", "sphere_colours", "cube_vertices",
                       "cube_colours")}
        ds = {n: v.data_ptr() for n, v in t.items()}
        ds.update(num_spheres=ns, num_cubes=nc)
        shape = (re - rb, w, 4) if args.format == "i32x4" else (re - rb, w)
        out = torch.empty(shape, dtype=torch.int32, device=dev)
        step = rt.bind_render_device(ds, w, h, (rb, re), out.data_ptr(), fmt=args.format,
                                     stream=stream.cuda_stream)
        ref = None
        for v in values:  # warmup + parity
            setter(v)
            for _ in range(3):
                step()
            torch.cuda.synchronize()
            if ref is None:
                ref = out.clone()
            elif not args.no_check and not torch.equal(out, ref):
                raise SystemExit(f"{cname}: {args.knob}={v} frame differs from {values[0]}")
        walls = {v: [] for v in values}
        kern = {v: {"prep_ms": [], "bin_ms": [], "trace_ms": []} for v in values}
        for _ in range(args.rounds):
            for v in values:
                setter(v)
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                for _ in range(args.steps):
                    step()
                torch.cuda.synchronize()
                walls[v].append((time.perf_counter() - t0) * 1e6 / args.steps)
                rt.profile(True)
                for _ in range(args.steps):
                    step()
                p = rt.profile_read()
                rt.profile(False)
                for key in kern[v]:
                    kern[v][key].append(p[key] * 1e3 / max(p["renders"], 1))
        step()
        res = {"config": cname, "knob": args.knob, "format": args.format, "fixed": args.fixed,
               "frame": f"{w}x{h} rows {rb}..{re}, {ns}+{nc}, seed {seed}, k {k}",
               "box_overdraw": round(rt.last_overdraw(), 3)}
        for v in values:
            res[str(v)] = {"wall_us": round(statistics.median(walls[v]), 1),
                           **{key.replace("_ms", "_us"): round(statistics.median(x), 1)
                              for key, x in kern[v].items()}}
        print(json.dumps(res), flush=True)
        del out, t
        torch.cuda.empty_cache()
    rt.close()


if __name__ == "__main__":
    main()
