#!/bin/bash
# Round 6: next-record scalar prefetch in trace_bin_kernel's walk
# (RT_REC_PREFETCH) against the shipped build, interleaved in one process,
# both formats, config 3 and config 3 sparse.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r06q; mkdir -p $O
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
V=opencl-ray-tracer_amd/variants
run() {  # name, args...
  local n=$1; shift
  timeout -k 10 300 python scripts/bench_variants.py $V/librt_hip_base.so $V/librt_hip_pf.so "$@" --kernels > $O/$n.json 2> $O/$n.err
  rc=$?; echo "$n rc=$rc"; python -c "
import json; d=json.load(open('$O/$n.json')); print({k: (v['prep_us'], v['bin_us'], v['trace_us'], v['median_us']) for k, v in d.items()})"
  grep -h MISMATCH $O/$n.err; [ $rc -ne 0 ] && { tail -20 $O/$n.err; exit $rc; }
}
run i32x4 --rounds 9
run rgba8 --format rgba8 --rounds 9
run sparse --k 1 --rounds 5
echo done
