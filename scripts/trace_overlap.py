"""Timeline of a rocprofv3 --kernel-trace run of the bench (frames in
flight): for the binned frames (prep -> coarse3 -> trace3 per frame), the
average kernel durations, how long consecutive trace kernels overlap, the
gap from one trace's end to the next trace's end (the steady-state frame
period) and how much of each frame's prep + coarse ran while another trace
was running.

    python scripts/trace_overlap.py gpurun_out/prof_x/run_kernel_trace.csv [--format i32x4|rgba8]
"""
import csv
import statistics
import sys


def main(path, fmt="i32x4"):
    rows = list(csv.DictReader(open(path)))
    tag = "trace3_kernel<0, 0>" if fmt == "i32x4" else "trace3_kernel<0, 1>"
    ks = []
    for r in rows:
        n = r["Kernel_Name"]
        kind = ("trace" if tag in n else "prep" if "prep_kernel" in n
                else "coarse" if "coarse3_kernel" in n else None)
        if kind:
            ks.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), kind,
                       r["Queue_Id"], n))
    ks.sort()
    traces = [k for k in ks if k[2] == "trace"]
    # runs of traces dispatched within 200 us of each other
    runs, cur = [], [traces[0]]
    for a, b in zip(traces, traces[1:]):
        if b[0] - a[1] < 200_000:
            cur.append(b)
        else:
            runs.append(cur)
            cur = [b]
    runs.append(cur)
    # frames in flight: the longest run that uses more than one queue
    multi = [r for r in runs if len({k[3] for k in r}) > 1 and len(r) >= 8]
    run = max(multi or runs, key=len)
    t0, t1 = run[0][0], run[-1][1]
    inside = [k for k in ks if t0 <= k[0] and k[1] <= t1]
    dur = {kind: statistics.mean((k[1] - k[0]) / 1e3 for k in inside if k[2] == kind)
           for kind in ("prep", "coarse", "trace")}
    ends = [k[1] for k in run]
    period = statistics.median((b - a) / 1e3 for a, b in zip(ends, ends[1:]))
    overlap = statistics.median(max(0, a[1] - b[0]) / 1e3 for a, b in zip(run, run[1:]))
    small = [k for k in inside if k[2] != "trace"]
    hidden = sum(sum(max(0, min(s[1], t[1]) - max(s[0], t[0])) for t in run)
                 for s in small) / max(1, sum(s[1] - s[0] for s in small))
    print(f"{fmt}: {len(run)} traces in the window, queues {sorted({k[3] for k in run})}")
    print("mean duration us: " + ", ".join(f"{k} {v:.1f}" for k, v in dur.items()))
    print(f"median trace-end to trace-end period {period:.1f} us; "
          f"median overlap of consecutive traces {overlap:.1f} us; "
          f"{100 * hidden:.0f} % of prep + coarse time ran beside a trace")


if __name__ == "__main__":
    fmt = "rgba8" if "--format" in sys.argv and sys.argv[sys.argv.index("--format") + 1] == "rgba8" else "i32x4"
    main(sys.argv[1], fmt)
