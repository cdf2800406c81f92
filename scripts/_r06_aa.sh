#!/bin/bash
# Round 6: RGBA8 tile pairs on one XCD (RT_RGBA8_PAIR_XCD: the two 16-pixel
# tiles sharing each 128-byte line written from one L2) against the shipped
# library, interleaved in one process: config 3 RGBA8 (coarse path,
# trace3_kernel), sparse RGBA8 (trace_bin_kernel), int32x4 (unchanged code,
# control); plus trace_bin's stores-only ablation with and without the pairs.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r06aa; mkdir -p $O
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
V=opencl-ray-tracer_amd/variants
run() {  # name, libs, args...
  local n=$1; local libs=$2; shift 2
  timeout -k 10 300 python scripts/bench_variants.py $libs "$@" --kernels > $O/$n.txt 2> $O/$n.err
  rc=$?; echo "$n rc=$rc"; grep -h MISMATCH $O/$n.txt; python -c "
import json; t=open('$O/$n.txt').read(); d=json.loads(t[t.index('{'):]); print({k: (v['prep_us'], v['bin_us'], v['trace_us'], v['median_us']) for k, v in d.items()})"
  [ $rc -ne 0 ] && { tail -20 $O/$n.err; exit $rc; }
}
run rgba8 "$V/librt_hip_base.so $V/librt_hip_px.so" --format rgba8 --rounds 9
run sparse_rgba8 "$V/librt_hip_base.so $V/librt_hip_px.so" --k 0.8 --format rgba8 --rounds 7
run i32x4 "$V/librt_hip_base.so $V/librt_hip_px.so" --rounds 5
run stores_rgba8 "$V/librt_hip_ab3.so $V/librt_hip_ab3px.so" --k 0.8 --format rgba8 --rounds 7
echo done
