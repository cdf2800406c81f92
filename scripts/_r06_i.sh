#!/bin/bash
# Round 6: (1) kernel-argument preloading into SGPRs (gfx950,
# -mllvm -amdgpu-kernarg-preload-count=16: a kernel's first 14 argument
# dwords arrive in user SGPRs); (2) the ballot walk in trace3_kernel with
# the list's first 64 entries loaded beside the count (RT_WALK_BALLOT=2)
# and without (=1); against the shipped build, interleaved in one process.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r06i; mkdir -p $O
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
V=opencl-ray-tracer_amd/variants
run() {  # name, args...
  local n=$1; shift
  timeout -k 10 300 python scripts/bench_variants.py "$@" --kernels > $O/$n.json 2> $O/$n.err
  rc=$?; echo "$n rc=$rc"; python -c "
import json; d=json.load(open('$O/$n.json')); print({k: (v['prep_us'], v['bin_us'], v['trace_us'], v['median_us']) for k, v in d.items()})"
  grep -h MISMATCH $O/$n.err; [ $rc -ne 0 ] && { tail -20 $O/$n.err; exit $rc; }
}
ALL="$V/librt_hip_base.so $V/librt_hip_kp.so $V/librt_hip_wb1.so $V/librt_hip_wb2.so"
run rgba8 $ALL --format rgba8 --rounds 9
run i32x4 $ALL --rounds 9
run i32x4_trace3 $V/librt_hip_base.so@trace_bin=2 $V/librt_hip_kp.so@trace_bin=2 $V/librt_hip_wb1.so@trace_bin=2 \
    $V/librt_hip_wb2.so@trace_bin=2 --rounds 7
run scene3 $ALL --scene 3 --rounds 9
run c5d_rgba8 $ALL --width 16384 --height 16384 --spheres 4096 --cubes 0 --seed 5 --rounds 5 --steps 10 --format rgba8
run c5d $ALL --width 16384 --height 16384 --spheres 4096 --cubes 0 --seed 5 --rounds 5 --steps 10
echo done
