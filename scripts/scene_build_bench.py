"""Scene build on the device (rt_scene_synthetic_device, SURVEY.md §8f row
f2) against the host build (rt_scene_synthetic) plus its upload, for the
BASELINE configs' synthetic scenes.  One JSON line per config.

    python scripts/scene_build_bench.py [--reps 50]
"""
import argparse
import json
import sys
import time
from pathlib import Path

import numpy as np

REPO = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(REPO))

CONFIGS = [("config2", 1920, 1080, 16, 4, 3.0), ("config3", 4096, 4096, 256, 64, 6.4),
           ("config4", 8192, 8192, 192, 64, 12.8), ("config5", 16384, 16384, 4096, 0, 25.6),
           ("large", 16384, 16384, 100000, 20000, 1.0)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=50)
    args = ap.parse_args()
    import torch
    import __graft_entry__
    pkg = __graft_entry__.load_package()
    dev = torch.device("cuda", 0)
    rt = pkg.RayTracer(0)
    stream = torch.cuda.Stream(dev)
    for name, w, h, n, m, k in CONFIGS:
        d = {"sphere_origins": torch.empty((n, 4), dtype=torch.float32, device=dev),
             "sphere_radius": torch.empty((n,), dtype=torch.float32, device=dev),
             "sphere_colours": torch.empty((n, 4), dtype=torch.float32, device=dev),
             "cube_vertices": torch.empty((m, 36, 4), dtype=torch.float32, device=dev),
             "cube_colours": torch.empty((m, 4), dtype=torch.float32, device=dev)}
        ptrs = {key: t.data_ptr() for key, t in d.items()}
        for _ in range(3):
            rt.scene_synthetic_device(w, h, n, m, 3, k, ptrs, stream=stream.cuda_stream)
        torch.cuda.synchronize(dev)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        for _ in range(args.reps):
            rt.scene_synthetic_device(w, h, n, m, 3, k, ptrs, stream=stream.cuda_stream)
        e1.record(stream)
        torch.cuda.synchronize(dev)
        dev_us = e0.elapsed_time(e1) * 1e3 / args.reps
        # host build + upload of the same arrays (the reference's path: build on
        # the host, copy on every trace, MainState.cpp:646-658, :755-816)
        host_reps = max(1, min(args.reps, 20))
        t0 = time.perf_counter()
        for _ in range(host_reps):
            s = pkg.Scene.synthetic(w, h, n, m, seed=3, k=k)
        build_us = (time.perf_counter() - t0) * 1e6 / host_reps
        t0 = time.perf_counter()
        for _ in range(host_reps):
            for key, t in d.items():
                t.copy_(torch.from_numpy(np.ascontiguousarray(getattr(s, key))))
            torch.cuda.synchronize(dev)
        upload_us = (time.perf_counter() - t0) * 1e6 / host_reps
        same = all(np.array_equal(t.cpu().numpy().view(np.uint32),
                                  np.ascontiguousarray(getattr(s, key)).view(np.uint32))
                   for key, t in d.items())
        # re-check the device build after the host copies overwrote the arrays
        rt.scene_synthetic_device(w, h, n, m, 3, k, ptrs, stream=stream.cuda_stream)
        torch.cuda.synchronize(dev)
        same = same and all(np.array_equal(t.cpu().numpy().view(np.uint32),
                                           np.ascontiguousarray(getattr(s, key)).view(np.uint32))
                            for key, t in d.items())
        nbytes = n * 36 + m * 592
        print(json.dumps({"scene": name, "spheres": n, "cubes": m, "bytes": nbytes,
                          "device_build_us": round(dev_us, 2),
                          "host_build_us": round(build_us, 1),
                          "host_upload_us": round(upload_us, 1), "bit_exact": bool(same)}),
              flush=True)
    rt.close()


if __name__ == "__main__":
    main()
