#!/bin/bash
# Round 6: the other BASELINE configs on the final library
# (scripts/other_configs.sh), then the LDS colour-table experiment
# (RT_COL_LDS) against the shipped build, interleaved in one process.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r06o; mkdir -p $O
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 900 bash scripts/other_configs.sh; rc=$?; cp gpurun_out/other_configs.jsonl $O/; [ $rc -ne 0 ] && exit $rc
V=opencl-ray-tracer_amd/variants
run() {  # name, args...
  local n=$1; shift
  timeout -k 10 300 python scripts/bench_variants.py $V/librt_hip_base.so $V/librt_hip_cl.so "$@" --kernels > $O/$n.json 2> $O/$n.err
  rc=$?; echo "$n rc=$rc"; python -c "
import json; d=json.load(open('$O/$n.json')); print({k: (v['prep_us'], v['bin_us'], v['trace_us'], v['median_us']) for k, v in d.items()})"
  grep -h MISMATCH $O/$n.err; [ $rc -ne 0 ] && { tail -20 $O/$n.err; exit $rc; }
}
run rgba8 --format rgba8 --rounds 9
run i32x4_trace3 --rounds 7 --format i32x4
echo done
