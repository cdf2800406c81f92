"""Per-launch durations of one kernel from a rocprofv3 --kernel-trace CSV
(run_kernel_trace.csv): count, mean, median, percentiles and the mean over
consecutive blocks of launches.  The --stats summary's AverageNs is the mean
over every launch of the command; for bench.py that includes the clock
ramps' first launches (at the idle clock) and the in-flight windows'
launches (two traces sharing the GPU), which pull the mean above the
steady one-stream duration the bench's profiled pass measures.

    python scripts/rocprof_launches.py run_kernel_trace.csv trace_bin_kernel
"""
import csv
import json
import statistics
import sys


def launches(path, name):
    rows = [r for r in csv.DictReader(open(path)) if name in r["Kernel_Name"]]
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    return [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in rows]


def summary(us, block=200):
    s = sorted(us)

    def pct(p):
        return s[min(len(s) - 1, int(p / 100 * len(s)))]
    return {"launches": len(us), "mean_us": round(statistics.mean(us), 2),
            "median_us": round(statistics.median(us), 2),
            "p5_us": round(pct(5), 2), "p95_us": round(pct(95), 2),
            "min_us": round(s[0], 2), "max_us": round(s[-1], 2),
            "block_means_us": [round(statistics.mean(us[i:i + block]), 1)
                               for i in range(0, len(us), block)]}


def main():
    path, name = sys.argv[1], sys.argv[2]
    out = {"file": path, "kernel": name, **summary(launches(path, name))}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
