"""Median kernel durations and inter-kernel gaps from a rocprofv3
kernel_trace.csv (one stream, frames of prep -> coarse -> trace)."""
import csv
import re
import statistics
import sys
from collections import defaultdict


def main(path):
    rows = list(csv.DictReader(open(path)))
    ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"])
                for r in rows)
    ev = [e for e in ev if any(k in e[2] for k in ("prep_kernel", "coarse3_kernel", "trace3_kernel"))]
    def short(n):
        return re.search(r"(prep_kernel|coarse3_kernel|trace3_kernel)", n).group(1)
    dur, gap = defaultdict(list), defaultdict(list)
    for a, b in zip(ev, ev[1:]):
        gap[f"{short(a[2])} -> {short(b[2])}"].append((b[0] - a[1]) / 1e3)
    for e in ev:
        dur[short(e[2])].append((e[1] - e[0]) / 1e3)
    frames = [(b[1] - a[0]) / 1e3 for a, b in zip(ev, ev[2:])
              if "prep" in a[2] and "trace3" in b[2]]
    for k, v in dur.items():
        print(f"{k:16s} n={len(v):4d} median {statistics.median(v):7.2f} us")
    for k, v in gap.items():
        print(f"gap {k:34s} n={len(v):4d} median {statistics.median(v):6.2f} us  min {min(v):6.2f}")
    if frames:
        print(f"prep start -> trace end: median {statistics.median(frames):.2f} us")


if __name__ == "__main__":
    main(sys.argv[1])
