"""Per-launch HBM traffic of the trace kernel from scripts/pmc.sh's passes 1
(WRITE_SIZE) and 2 (FETCH_SIZE), corrected as MI355X_MICROARCH.md's
HBM/rocprofv3 section prescribes (KB units; FETCH_SIZE doubled on gfx950).
Writes the JSON bench.py reads `roofline.traffic` from.

    python scripts/pmc_traffic.py gpurun_out/pmc_r01 profiles/r01_pmc_config3.json
    python scripts/pmc_traffic.py gpurun_out/pmc_c4 profiles/r04/pmc_config4.json 8192 8192 192 64 4 i32x4
"""
import csv
import json
import re
import sys

KERNEL = re.compile(r"trace\d?_kernel<0(, 0)?>|trace_bin_kernel<0>")


def per_launch(path, counter):
    """The counter per launch of the bench's dominant trace kernel: of the
    kernels matching KERNEL, the one launched most often (the automatic path
    choice runs trace3_kernel on a context's first frame, trace_bin_kernel
    after it)."""
    by = {}
    for r in csv.DictReader(open(path)):
        m = KERNEL.search(r["Kernel_Name"])
        if m and r["Counter_Name"] == counter:
            by.setdefault(m.group(0), []).append(float(r["Counter_Value"]))
    if not by:
        raise SystemExit(f"no {counter} rows for the trace kernel in {path}")
    name, vals = max(by.items(), key=lambda kv: len(kv[1]))
    return sum(vals) / len(vals), len(vals), name


def main(prefix, out, config=(4096, 4096, 256, 64, 3, "i32x4")):
    w_kb, nw, kname = per_launch(f"{prefix}_1/run_counter_collection.csv", "WRITE_SIZE")
    f_kb, nf, _ = per_launch(f"{prefix}_2/run_counter_collection.csv", "FETCH_SIZE")
    write_b = int(round(w_kb * 1024))
    fetch_b = int(round(f_kb * 1024 * 2))
    w, h = int(config[0]), int(config[1])
    algo = w * h * (16 if config[5] == "i32x4" else 4)
    d = {"config": [w, h, int(config[2]), int(config[3]), int(config[4]), config[5]],
         "kernel": kname,
         "write_bytes_per_launch": write_b, "fetch_bytes_per_launch": fetch_b,
         "hbm_bytes_per_launch": write_b + fetch_b,
         "algo_bytes_per_launch": algo,
         "launches": [nw, nf],
         "method": "rocprofv3 --kernel-trace --pmc WRITE_SIZE and --pmc FETCH_SIZE in separate "
                   "runs of bench.py (scripts/pmc.sh, BENCH_ARGS); KB x 1024; "
                   "FETCH_SIZE doubled (gfx950 reports half of wide reads, "
                   "MI355X_MICROARCH.md)"}
    json.dump(d, open(out, "w"), indent=1)
    print(json.dumps(d))


if __name__ == "__main__":
    # optional: W H SPHERES CUBES SEED FORMAT of the run (default config 3)
    main(sys.argv[1], sys.argv[2], *([tuple(sys.argv[3:9])] if len(sys.argv) >= 9 else []))
