"""Frames in flight on CU-masked streams: K renders of the bench's config-3
frame spread round-robin over S (context, stream, frame) slots whose streams
are created with hipExtStreamCreateWithCUMask, so one slot's small prep /
coarse kernels find free CUs while the other slot's trace runs.  Each mask
is a 32-bit pattern repeated over the CU mask words (every 32-CU group gets
the same share).  Prints us per frame per setting; every slot's frame is
checked bit-exact against a plain single-stream render.

    python scripts/inflight_cumask.py --settings "1:ffffffff" "2:ffffffff,ffffffff" \
        "2:0000ffff,ffff0000" "2:00ffffff,ffffff00"
"""
import argparse
import ctypes
import statistics
import sys
import time
from pathlib import Path

import numpy as np

REPO = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(REPO))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--settings", nargs="+",
                    default=["1:ffffffff", "2:ffffffff,ffffffff", "2:0000ffff,ffff0000"])
    ap.add_argument("--rounds", type=int, default=7)
    ap.add_argument("--steps", type=int, default=40)
    ap.add_argument("--size", type=int, default=4096)
    ap.add_argument("--format", default="i32x4", choices=("i32x4", "rgba8"))
    ap.add_argument("--spheres", type=int, default=256)
    ap.add_argument("--cubes", type=int, default=64)
    ap.add_argument("--seed", type=int, default=3)
    args = ap.parse_args()
    import torch
    import __graft_entry__
    pkg = __graft_entry__.load_package()
    hip = ctypes.CDLL("libamdhip64.so")
    hip.hipExtStreamCreateWithCUMask.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_uint32,
                                                 ctypes.POINTER(ctypes.c_uint32)]
    n_cu = torch.cuda.get_device_properties(0).multi_processor_count
    words = (n_cu + 31) // 32
    w = h = args.size
    scene = pkg.Scene.synthetic(w, h, args.spheres, args.cubes, seed=args.seed, k=w / 640)
    dev = torch.device("cuda:0")
    t = {n: torch.from_numpy(np.ascontiguousarray(getattr(scene, n))).to(dev)
         for n in ("sphere_origins", "sphere_radius", "sphere_colours", "cube_vertices",
                   "cube_colours")}
    ds = {n: v.data_ptr() for n, v in t.items()}
    ds["num_spheres"], ds["num_cubes"] = scene.num_spheres, scene.num_cubes
    shape = (h, w, 4) if args.format == "i32x4" else (h, w)
    ref_out = torch.empty(shape, dtype=torch.int32, device=dev)
    rt0 = pkg.RayTracer(0)
    s0 = torch.cuda.Stream(dev)
    rt0.bind_render_device(ds, w, h, (0, h), ref_out.data_ptr(), fmt=args.format,
                           stream=s0.cuda_stream)()
    torch.cuda.synchronize()
    ref = ref_out.cpu()
    setups = []
    for spec in args.settings:
        n, masks = spec.split(":")
        pats = [int(m, 16) for m in masks.split(",")]
        assert len(pats) == int(n)
        fns, outs, keep = [], [], []
        for p in pats:
            st = ctypes.c_void_p()
            arr = (ctypes.c_uint32 * words)(*([p] * words))
            assert hip.hipExtStreamCreateWithCUMask(ctypes.byref(st), words, arr) == 0
            rt = pkg.RayTracer(0)
            out = torch.empty(shape, dtype=torch.int32, device=dev)
            fns.append(rt.bind_render_device(ds, w, h, (0, h), out.data_ptr(), fmt=args.format,
                                             stream=st.value))
            outs.append(out)
            keep.append((rt, st))
        setups.append((spec, fns, outs, keep))
    res = {spec: [] for spec, *_ in setups}
    for r in range(args.rounds):
        for spec, fns, outs, _ in setups:
            s = len(fns)
            for i in range(4 * s):
                fns[i % s]()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for i in range(args.steps):
                fns[i % s]()
            torch.cuda.synchronize()
            res[spec].append((time.perf_counter() - t0) / args.steps * 1e6)
    for spec, fns, outs, _ in setups:
        for o in outs:
            assert torch.equal(o.cpu(), ref), f"{spec}: frame differs"
        med = statistics.median(res[spec])
        print(f"{spec:28s} {med:7.1f} us/frame  {w * h / med / 1e3:6.1f} Grays/s  "
              f"(min {min(res[spec]):.1f})", flush=True)


if __name__ == "__main__":
    main()
