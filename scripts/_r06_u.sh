#!/bin/bash
# Round 6: trace_bin_kernel's prologue.  base = shipped; mf = the bin's mask
# words loaded before the non-finite flag is tested (a build knob while
# measured, RT_BIN_MASK_FIRST; not kept: profiles/r06/bin_prologue/mask_first.patch);
# ra = arguments reordered so the flag pointer, the mask pointers and the
# sizes are in the 14 preloaded dwords (kept); mfa = both.  Interleaved in one
# process, config 3 int32x4, config 3 sparse (int32x4, RGBA8 below 1 frame).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r06u; mkdir -p $O
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
V=opencl-ray-tracer_amd/variants
run() {  # name, args...
  local n=$1; shift
  timeout -k 10 300 python scripts/bench_variants.py $V/librt_hip_base.so $V/librt_hip_mf.so $V/librt_hip_ra.so $V/librt_hip_mfa.so "$@" --kernels > $O/$n.json 2> $O/$n.err
  rc=$?; echo "$n rc=$rc"; python -c "
import json; d=json.load(open('$O/$n.json')); print({k: (v['prep_us'], v['bin_us'], v['trace_us'], v['median_us']) for k, v in d.items()})"
  grep -h MISMATCH $O/$n.err; [ $rc -ne 0 ] && { tail -20 $O/$n.err; exit $rc; }
}
run i32x4 --rounds 9
run sparse --k 1 --rounds 7
run sparse_rgba8 --k 0.8 --format rgba8 --rounds 7
echo done
