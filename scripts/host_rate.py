"""Is the Python frame loop host-bound?  (round 5)  For config 3 with S slots
on CU-masked streams (the bench's in-flight loop): the host time of one
step() (enqueue only) and the loop's time per frame for K = 20 and K = 200
frames; the C++ rt_headless --throughput loop is the comparison."""
import statistics
import sys
import time
from pathlib import Path

REPO = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(REPO))


def main():
    import torch
    import __graft_entry__
    import bench
    pkg = __graft_entry__.load_package()
    args = bench.parse([])
    c = bench.Ctx(args)
    w = h = 4096
    scene, ds = bench.device_scene(pkg, c, w, h, 256, 64, 3, w / 640)
    for fmt, slots in (("i32x4", 2), ("i32x4", 1), ("rgba8", 3)):
        step, frames, keep = bench.inflight_step(pkg, c, ds, w, h, fmt, "auto", slots)
        for _ in range(200):
            step()
        torch.cuda.synchronize()
        # host enqueue time per step: 8 steps at a time, then drain
        host = []
        for _ in range(20):
            t0 = time.perf_counter()
            for _ in range(8):
                step()
            host.append((time.perf_counter() - t0) / 8 * 1e6)
            torch.cuda.synchronize()
        res = {}
        for k in (20, 200):
            per = []
            for _ in range(5):
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                for _ in range(k):
                    step()
                torch.cuda.synchronize()
                per.append((time.perf_counter() - t0) / k * 1e6)
            res[k] = statistics.median(per)
        print(f"{fmt} {slots} slots: host enqueue {statistics.median(host):.1f} us/step; "
              f"loop K=20 {res[20]:.1f} us/frame, K=200 {res[200]:.1f} us/frame", flush=True)
        torch.cuda.synchronize()
        for rt in keep[0]:
            rt.close()
        if isinstance(keep[1], bench.HipStreams):
            keep[1].close()


if __name__ == "__main__":
    main()
