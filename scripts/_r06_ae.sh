#!/bin/bash
# Round 6: spheres whose disc no pixel of the wave reaches skip their square
# roots with one ballot (RT_SPH_SKIP_MISS) against the shipped library,
# interleaved in one process: config 3 both formats, sparse.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r06ae; mkdir -p $O
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
V=opencl-ray-tracer_amd/variants
run() {  # name, args...
  local n=$1; shift
  timeout -k 10 300 python scripts/bench_variants.py $V/librt_hip_base.so $V/librt_hip_sk.so "$@" --kernels > $O/$n.txt 2> $O/$n.err
  rc=$?; echo "$n rc=$rc"; grep -h MISMATCH $O/$n.txt; python -c "
import json; t=open('$O/$n.txt').read(); d=json.loads(t[t.index('{'):]); print({k: (v['prep_us'], v['trace_us'], v['median_us']) for k, v in d.items()})"
  [ $rc -ne 0 ] && { tail -20 $O/$n.err; exit $rc; }
}
run i32x4 --rounds 9
run rgba8 --format rgba8 --rounds 9
run sparse --k 1 --rounds 7
run sparse_rgba8 --k 0.8 --format rgba8 --rounds 7
echo done
