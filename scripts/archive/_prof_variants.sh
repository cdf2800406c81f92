#!/bin/bash
# rocprofv3 kernel stats of each variant library on config 3 (one run each).
set -e
R="${GRAFT_REPO_ROOT:-$(pwd)}"; V=$R/opencl-ray-tracer_amd/variants
mkdir -p $R/gpurun_out; export TMPDIR=/tmp
EXTRA=${EXTRA:-}
for v in "$@"; do
  (cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/pv_$v -o run --output-format csv -- \
     python $R/scripts/bench_variants.py $V/librt_hip_$v.so --rounds 3 $EXTRA > $R/gpurun_out/pv_$v.log 2>&1)
  echo "== $v"; python3 - "$R/gpurun_out/pv_$v" <<'PY'
import csv,glob,sys
f=glob.glob(sys.argv[1]+"/**/run_kernel_stats.csv",recursive=True)[0]
for r in csv.DictReader(open(f)):
    n=r["Name"]; n=n[n.find("::")+2:][:40] if "::" in n else n[:40]
    print(f'{n:42s} calls {r["Calls"]:>5} avg_us {float(r["AverageNs"])/1e3:8.2f}')
PY
done
