#!/bin/bash
# Round 6: trace_bin_kernel's walk taken apart (diagnostic builds, frames
# wrong on purpose): RT_BIN_ABLATE 1 = no walk; 4 = the walk without the
# hit-colour gather; 5 = the walk's record loads without the exact tests
# (so no gather either); against the shipped library, interleaved in one
# process; config 3 int32x4 and sparse RGBA8.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r06ad; mkdir -p $O
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
V=opencl-ray-tracer_amd/variants
run() {  # name, args...
  local n=$1; shift
  timeout -k 10 300 python scripts/bench_variants.py $V/librt_hip_base.so $V/librt_hip_ab1.so $V/librt_hip_ab4.so $V/librt_hip_ab5.so "$@" --kernels > $O/$n.txt 2> $O/$n.err
  rc=$?; echo "$n rc=$rc"; python -c "
import json; t=open('$O/$n.txt').read(); d=json.loads(t[t.index('{'):]); print({k: (v['trace_us'], v['median_us']) for k, v in d.items()})"
  [ $rc -ne 0 ] && { tail -20 $O/$n.err; exit $rc; }
}
run i32x4 --rounds 9
run sparse_rgba8 --k 0.8 --format rgba8 --rounds 9
echo done
