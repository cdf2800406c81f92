"""Frames in flight on CU-masked slot streams (round 5): every slot on every
CU (the bench's default) against slots on disjoint CU sets -- whole XCDs
(contiguous halves of the mask) or alternate CUs.  Config 3's frame, both
formats; every slot's frame checked bit-exact."""
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
    ap.add_argument("--format", default="i32x4", choices=("i32x4", "rgba8"))
    ap.add_argument("--slots", type=int, default=2)
    ap.add_argument("--rounds", type=int, default=7)
    ap.add_argument("--steps", type=int, default=40)
    args = ap.parse_args()
    import torch
    import __graft_entry__
    import bench
    pkg = __graft_entry__.load_package()
    w = h = 4096
    scene = pkg.Scene.synthetic(w, h, 256, 64, seed=3, k=w / 640)
    dev = torch.device("cuda:0")
    t = {n: torch.from_numpy(np.ascontiguousarray(getattr(scene, n))).to(dev)
         for n in ("sphere_origins", "sphere_radius", "sphere_colours", "cube_vertices",
                   "cube_colours")}
    ds = {n: v.data_ptr() for n, v in t.items()}
    ds["num_spheres"], ds["num_cubes"] = scene.num_spheres, scene.num_cubes
    n_cu = torch.cuda.get_device_properties(dev).multi_processor_count
    nw = (n_cu + 31) // 32
    S = args.slots

    def mask_of(cus):
        words = [0] * nw
        for c in cus:
            words[c // 32] |= 1 << (c % 32)
        return words
    layouts = {
        "all": [mask_of(range(n_cu))] * S,
        "contiguous": [mask_of(range(k * n_cu // S, (k + 1) * n_cu // S)) for k in range(S)],
        "alternate": [mask_of(range(k, n_cu, S)) for k in range(S)],
    }
    shape = (h, w, 4) if args.format == "i32x4" else (h, w)
    ref = None
    res = {k: [] for k in layouts}
    setups = {}
    for name, masks in layouts.items():
        st = bench.HipStreams(S, nw, masks)
        rts = [pkg.RayTracer(0) for _ in range(S)]
        outs = [torch.empty(shape, dtype=torch.int32, device=dev) for _ in range(S)]
        fns = [rt.bind_render_device(ds, w, h, (0, h), o.data_ptr(), fmt=args.format, stream=s)
               for rt, o, s in zip(rts, outs, st.handles)]
        setups[name] = (st, rts, outs, fns)
    for r in range(args.rounds):
        for name, (st, rts, outs, fns) in setups.items():
            for i in range(4 * S):
                fns[i % S]()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for i in range(args.steps):
                fns[i % S]()
            torch.cuda.synchronize()
            res[name].append((time.perf_counter() - t0) / args.steps * 1e6)
            if ref is None:
                ref = outs[0].clone()
            for o in outs:
                assert torch.equal(o, ref), name
    for name, v in res.items():
        print(f"{args.format} {S} slots, CUs {name}: {statistics.median(v):.1f} us/frame "
              f"(min {min(v):.1f})", flush=True)
    for st, rts, outs, fns in setups.values():
        for rt in rts:
            rt.close()
        st.close()


if __name__ == "__main__":
    main()
