"""Where the first rt_render's kernel time goes: in a
fresh process, reference scene 1 at 640x480 through rt_render, per call the
event interval kernel_us (ev[1] -> ev[2], what rt_timing reports) beside the
kernels' own durations (rt_profile: events on each kernel's dispatch
packet).  A gap between the two on the first call is host-side enqueue
latency; equal values mean the kernels themselves ran slower (cold caches,
clocks).

    python scripts/first_call.py [--calls 6] [--idle-ms 0]
"""
import argparse
import json
import sys
import time
from pathlib import Path

import numpy as np

REPO = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(REPO))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--calls", type=int, default=6)
    ap.add_argument("--idle-ms", type=float, default=0.0, help="sleep between calls")
    ap.add_argument("--scene", type=int, default=1)
    ap.add_argument("--warm-d2h", type=int, default=0,
                    help="bytes of a pageable device-to-host copy (torch) before rt_init")
    ap.add_argument("--reserve", action="store_true", help="rt_reserve before the first call")
    args = ap.parse_args()
    import __graft_entry__
    pkg = __graft_entry__.load_package()
    if args.warm_d2h:
        import torch
        torch.zeros(args.warm_d2h // 4, dtype=torch.int32, device="cuda:0").cpu()
        torch.cuda.synchronize()
    with np.load(REPO / "tests" / "golden" / f"scene{args.scene}_640x480.npz") as z:
        g = {k: z[k] for k in z.files}
    scene = pkg.Scene(g["sphere_origins"], g["sphere_radius"], g["sphere_colours"],
                      g["cube_vertices"], g["cube_colours"])
    out = np.zeros((480, 640, 4), np.int32)
    t0 = time.perf_counter()
    rt = pkg.RayTracer(0)
    init_ms = (time.perf_counter() - t0) * 1e3
    if args.reserve:
        rt.reserve(640, 480, scene.num_spheres, scene.num_cubes)
    rows = []
    for i in range(args.calls):
        _, t = rt.render(scene, 640, 480, out=out)  # kernel_us: the kernels' own span
        rt.profile(True)
        rt.render(scene, 640, 480, out=out)  # each kernel's own duration, summed
        p = rt.profile_read()
        rt.profile(False)
        rows.append({"call": i, "kernel_us": round(t.kernel_us, 1),
                     "kernels_own_us": round(1e3 * (p["prep_ms"] + p["bin_ms"] + p["trace_ms"]), 1),
                     "total_us": round(t.total_us, 1), "download_us": round(t.download_us, 1),
                     "ok": bool(np.array_equal(out, g["frame"])), "kernel": rt.last_kernel()})
        if args.idle_ms:
            time.sleep(args.idle_ms / 1e3)
    rt.close()
    print(json.dumps({"init_ms": round(init_ms, 2), "calls": rows}))


if __name__ == "__main__":
    main()
