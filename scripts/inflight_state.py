"""Why is bench.py's in-flight loop slower than the same loop in a fresh
process?  (round 5)  Config 3, int32x4, 2 slots on CU-masked streams: the
loop's time per frame (median of reps, K = 20 and K = 200) measured fresh,
then again after each phase bench.py runs before its in-flight loop, in
bench.py's order: the app workload (measure_app), the one-stream context's
warmup + clock ramp, the one-stream K loop with torch timing events, the
profiled-event pass."""
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

    def measure(label):
        step, frames, keep = bench.inflight_step(pkg, c, ds, w, h, "i32x4", "auto", 2)
        for _ in range(13):
            step()
        c.sync()
        res = {}
        for k, reps in ((20, 7), (200, 3)):
            res[k] = statistics.median(c.timed(step, k) * 1e3 for _ in range(reps))
        c.sync()
        for rt in keep[0]:
            rt.close()
        keep[1].close()
        print(f"{label:28s} K=20 {res[20]:.1f} us/frame  K=200 {res[200]:.1f} us/frame",
              flush=True)

    measure("fresh")
    measure("fresh again")
    bench.measure_app(args, c, pkg)
    measure("after measure_app")
    rt = pkg.RayTracer(c.gpu)
    out = bench.frame_tensor(c, h, w, "i32x4")
    step = rt.bind_render_device(ds, w, h, (0, h), out.data_ptr(), fmt="i32x4", path="auto",
                                 stream=c.stream.cuda_stream)
    for _ in range(5):
        step()
    c.clock_ramp(step, 50.0)
    c.sync()
    measure("after one-stream ramp")
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    c.timed(step, 20, events=(ev0, ev1))
    measure("after torch timing events")
    rt.profile(True)
    for _ in range(20):
        step()
    c.sync()
    rt.profile_read()
    rt.profile(True)
    c.timed(step, 20)
    rt.profile_read()
    rt.profile(False)
    measure("after profiled pass")
    rt.close()
    measure("after closing the context")
    time.sleep(0.5)
    measure("after 0.5 s idle")


if __name__ == "__main__":
    main()
