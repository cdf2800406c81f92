"""Frames in flight: K renders of the bench's config-3 frame spread round-robin
over S (context, stream, frame buffer) slots, S = 1, 2, 3, interleaved
rounds; prints µs per frame.  Every slot's frame is checked bit-exact
against the single-stream frame."""
import argparse
import statistics
import sys
import time
from pathlib import Path

import numpy as np

REPO = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(REPO))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--slots", default="1,2,3")
    ap.add_argument("--rounds", type=int, default=7)
    ap.add_argument("--steps", type=int, default=40)
    ap.add_argument("--size", type=int, default=4096)
    ap.add_argument("--format", default="i32x4", choices=("i32x4", "rgba8"))
    ap.add_argument("--k", type=float, default=None, help="object scale (default W/640: dense)")
    ap.add_argument("--knob", default=None,
                    help="RayTracer setter (without set_) applied to every slot, e.g. coarse_lds")
    ap.add_argument("--values", default="0", help="the knob's settings, interleaved")
    ap.add_argument("--fixed", action="append", default=[],
                    help="knob=value held on every slot for every setting (repeatable)")
    args = ap.parse_args()
    import torch
    import __graft_entry__
    pkg = __graft_entry__.load_package()
    w = h = args.size
    scene = pkg.Scene.synthetic(w, h, 256, 64, seed=3, k=args.k if args.k is not None else w / 640)
    dev = torch.device("cuda:0")
    t = {n: torch.from_numpy(np.ascontiguousarray(getattr(scene, n))).to(dev)
         for n in ("sphere_origins", "sphere_radius", "sphere_colours", "cube_vertices",
                   "cube_colours")}
    ds = {n: v.data_ptr() for n, v in t.items()}
    ds["num_spheres"], ds["num_cubes"] = scene.num_spheres, scene.num_cubes
    slots = [int(s) for s in args.slots.split(",")]
    smax = max(slots)
    ctxs = [pkg.RayTracer(0) for _ in range(smax)]
    streams = [torch.cuda.Stream(dev) for _ in range(smax)]
    shape = (h, w, 4) if args.format == "i32x4" else (h, w)
    outs = [torch.empty(shape, dtype=torch.int32, device=dev) for _ in range(smax)]
    fns = [ctxs[i].bind_render_device(ds, w, h, (0, h), outs[i].data_ptr(), fmt=args.format,
                                      stream=streams[i].cuda_stream) for i in range(smax)]
    for kv in args.fixed:
        name, val = kv.split("=")
        for c in ctxs:
            getattr(c, "set_" + name)(int(val))
    values = [int(v) for v in args.values.split(",")]
    res = {(v, s): [] for v in values for s in slots}
    ref = None
    for r in range(args.rounds):
        for v in values:
            if args.knob == "trace_path":  # as scripts/ab_knob.py
                for c in ctxs:
                    c.set_trace_bin({0: 2, 1: 1}[v])
            elif args.knob:
                for c in ctxs:
                    getattr(c, "set_" + args.knob)(v)
            for s in slots:
                for i in range(2 * s):
                    fns[i % s]()
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                for i in range(args.steps):
                    fns[i % s]()
                torch.cuda.synchronize()
                res[(v, s)].append((time.perf_counter() - t0) / args.steps * 1e6)
                if ref is None:
                    ref = outs[0].cpu()
                for i in range(s):
                    assert torch.equal(outs[i].cpu(), ref), f"slot {i} differs ({args.knob}={v})"
    for v in values:
        for s in slots:
            med = statistics.median(res[(v, s)])
            print(f"{args.format} {args.knob}={v} slots {s}: {med:.1f} us/frame  "
                  f"{w * h / med / 1e3:.1f} Grays/s  (min {min(res[(v, s)]):.1f})")


if __name__ == "__main__":
    main()
