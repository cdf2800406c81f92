#!/bin/bash
# Round 6: where trace_bin_kernel's time goes at config 3 (diagnostic builds,
# frames wrong on purpose: RT_BIN_ABLATE 1 = no walk, 2 = no classification
# either, 3 = no mask loads either, stores of the background only), against
# the shipped library, interleaved in one process; int32x4 and sparse RGBA8.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r06z; mkdir -p $O
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
V=opencl-ray-tracer_amd/variants
run() {  # name, args...
  local n=$1; shift
  timeout -k 10 300 python scripts/bench_variants.py $V/librt_hip_base.so $V/librt_hip_ab1.so $V/librt_hip_ab2.so $V/librt_hip_ab3.so "$@" --kernels > $O/$n.json 2> $O/$n.err
  rc=$?; echo "$n rc=$rc"; python -c "
import json; d=json.load(open('$O/$n.json')); print({k: (v['prep_us'], v['trace_us'], v['median_us']) for k, v in d.items()})"
  [ $rc -ne 0 ] && { tail -20 $O/$n.err; exit $rc; }
}
run i32x4 --rounds 7
run sparse_rgba8 --k 0.8 --format rgba8 --rounds 7
echo done
