"""Where the bench's K-frame window loses time against the long window
(round 6).  Config 3, int32x4, 2 slots on CU-masked streams, after the
bench's clock ramp: (1) the window's wall time for K = 5 ... 200 (median of
reps), fitted as a + b K (a = what one window pays once); (2) one K = 20
window with an event after every frame on its slot's stream: each frame's
completion time from an event recorded on slot 0's stream before frame 0,
against the wall clock around the window."""
import json
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
    fmt = sys.argv[1] if len(sys.argv) > 1 else "i32x4"
    slots = 2 if fmt == "i32x4" else 3
    scene, ds = bench.device_scene(pkg, c, w, h, 256, 64, 3, w / 640)
    step, frames, keep = bench.inflight_step(pkg, c, ds, w, h, fmt, "auto", slots)
    for _ in range(4 * slots + 5):
        step()
    c.sync()
    out = {"format": fmt, "slots": slots, "window_us_per_frame": {}}
    ks = (5, 10, 20, 40, 100, 200)
    for k in ks:
        c.clock_ramp(step, 50.0)
        out["window_us_per_frame"][k] = round(statistics.median(
            c.timed(step, k) * 1e3 for _ in range(5)), 2)
    tot = [out["window_us_per_frame"][k] * k for k in ks]
    n = len(ks)
    mk, mt = sum(ks) / n, sum(tot) / n
    b = sum((k - mk) * (t - mt) for k, t in zip(ks, tot)) / sum((k - mk) ** 2 for k in ks)
    out["fit"] = {"a_us": round(mt - b * mk, 1), "b_us_per_frame": round(b, 2)}
    # one K = 20 window with per-frame events
    handles = keep[1].handles
    ext = [torch.cuda.ExternalStream(hd, device=c.dev) for hd in handles]
    runs = []
    for rep in range(5):
        c.clock_ramp(step, 50.0)
        # the next step() renders on slot keep-cycle position: find it
        ev0 = torch.cuda.Event(enable_timing=True)
        evs = [torch.cuda.Event(enable_timing=True) for _ in range(20)]
        c.sync()
        t0 = time.perf_counter()
        ev0.record(ext[0])
        enq = []
        for i in range(20):
            step()
            enq.append((time.perf_counter() - t0) * 1e6)
            # the frame just enqueued went to the slot before the counter
            evs[i].record(ext[(keep_slot(step) - 1) % slots])
        c.sync()
        wall = (time.perf_counter() - t0) * 1e6
        done = [round(ev0.elapsed_time(e) * 1e3, 1) for e in evs]
        runs.append({"wall_us": round(wall, 1), "done_us": done,
                     "enqueued_us": [round(x, 1) for x in enq]})
    out["k20_timelines"] = runs
    # what one synchronisation costs on an idle GPU: torch's device-wide sync
    # (the bench's), one slot stream's, and a recorded event's
    import ctypes
    hip = ctypes.CDLL("libamdhip64.so")
    hip.hipStreamSynchronize.argtypes = [ctypes.c_void_p]
    c.sync()

    def idle(fn, n=200):
        ts = []
        for _ in range(n):
            t = time.perf_counter()
            fn()
            ts.append((time.perf_counter() - t) * 1e6)
        return round(statistics.median(ts), 2)
    ev = torch.cuda.Event()
    ev.record(ext[0])
    out["idle_sync_us"] = {"torch.cuda.synchronize": idle(c.sync),
                           "hipStreamSynchronize(slot 0)": idle(lambda: hip.hipStreamSynchronize(handles[0])),
                           "event.synchronize": idle(ev.synchronize)}
    # and after a frame: enqueue one, wait for it by each method
    def after_frame(waiter, n=20):
        ts = []
        for _ in range(n):
            c.sync()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            slot = keep_slot(step) % slots
            e0.record(ext[slot])
            t = time.perf_counter()
            step()
            e1.record(ext[slot])
            waiter(slot)
            wall = (time.perf_counter() - t) * 1e6
            ts.append(wall - e0.elapsed_time(e1) * 1e3)
        return round(statistics.median(ts), 2)
    out["one_frame_wall_minus_gpu_us"] = {
        "torch.cuda.synchronize": after_frame(lambda s: c.sync()),
        "hipStreamSynchronize": after_frame(lambda s: hip.hipStreamSynchronize(handles[s]))}
    print(json.dumps(out))


def keep_slot(step):
    """Frames enqueued so far: inflight_step's counter, the one-int list in
    step()'s closure."""
    for cell in step.__closure__:
        v = cell.cell_contents
        if isinstance(v, list) and len(v) == 1 and isinstance(v[0], int):
            return v[0]
    raise RuntimeError("no frame counter in step()")


if __name__ == "__main__":
    main()
