#!/bin/bash
# Round 3: HBM traffic per trace launch of config 5 dense with nontemporal
# stores (wide build): WRITE_SIZE and FETCH_SIZE in separate rocprofv3 passes.
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
ARGS="--width 16384 --height 16384 --spheres 4096 --cubes 0 --seed 5 --steps 5 --warmup 2 --inflight 1 --no-extras --no-cpu-baseline --no-host-path"
i=0
for grp in WRITE_SIZE FETCH_SIZE; do
  i=$((i+1))
  (cd /tmp && timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $grp -d "$R/gpurun_out/pmc_c5d_$i" -o run --output-format csv -- \
      python "$R/bench.py" $ARGS > "$R/gpurun_out/pmc_c5d_$i.log" 2>&1)
  rc=$?; echo "pmc pass $i ($grp) rc=$rc"; [ $rc -ne 0 ] && { tail -8 "$R/gpurun_out/pmc_c5d_$i.log"; exit $rc; }
done
python - <<'PY'
import csv, json, re
K = re.compile(r"trace3_kernel<0, 0>")
def avg(p, c):
    v = [float(r["Counter_Value"]) for r in csv.DictReader(open(p)) if K.search(r["Kernel_Name"]) and r["Counter_Name"] == c]
    return sum(v) / len(v), len(v)
w, nw = avg("gpurun_out/pmc_c5d_1/run_counter_collection.csv", "WRITE_SIZE")
f, nf = avg("gpurun_out/pmc_c5d_2/run_counter_collection.csv", "FETCH_SIZE")
d = {"config": [16384, 16384, 4096, 0, 5, "i32x4", "dense"], "kernel": "wide::trace3_kernel<0, 0> (nontemporal stores)",
     "write_bytes_per_launch": int(w * 1024), "fetch_bytes_per_launch": int(f * 1024 * 2),
     "algo_bytes_per_launch": 16384 * 16384 * 16, "launches": [nw, nf],
     "method": "rocprofv3 --kernel-trace --pmc WRITE_SIZE / FETCH_SIZE, separate runs; KB x 1024; FETCH_SIZE doubled (gfx950)"}
d["hbm_over_algo"] = round((d["write_bytes_per_launch"] + d["fetch_bytes_per_launch"]) / d["algo_bytes_per_launch"], 4)
json.dump(d, open("gpurun_out/pmc_c5d_nt.json", "w"), indent=1); print(json.dumps(d))
PY
