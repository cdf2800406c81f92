#!/bin/bash
# Round 5: trace_bin_kernel with the classifier load beside the box load
# (RT_TBIN_HOIST) against the merged build; then PMC traffic / mix of the
# merged build's bench (the trace_bin_kernel headline).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r05h; mkdir -p $O
V=opencl-ray-tracer_amd/variants
for f in i32x4 rgba8; do
  timeout -k 10 300 python scripts/bench_variants.py $V/librt_hip_base.so@trace_bin=1 $V/librt_hip_hoist.so@trace_bin=1 \
      --format $f --kernels > $O/ab_$f.json 2>$O/ab_$f.err
  rc=$?; echo "ab $f rc=$rc"; cat $O/ab_$f.json; [ $rc -ne 0 ] && { tail -3 $O/ab_$f.err; exit $rc; }
done
TAG=r05 BENCH_ARGS="--steps 10 --warmup 3 --no-cpu-baseline --no-host-path" bash scripts/pmc.sh > $O/pmc.log 2>&1
rc=$?; tail -8 $O/pmc.log; [ $rc -ne 0 ] && exit $rc
python scripts/pmc_traffic.py gpurun_out/pmc_r05 $O/r05_pmc_config3.json
# the no-coarse crossover by box overdraw, both formats
for f in rgba8 i32x4; do
  timeout -k 10 300 python scripts/ab_knob.py --knob trace_path --values 0,1 --format $f \
      --configs c3s,c3r2,c3r3,c3r45,c3,c3r8,c3k15 2>&1 | grep -v amdgpu.ids > $O/cross_$f.jsonl
  rc=${PIPESTATUS[0]}; echo "cross $f rc=$rc"; cat $O/cross_$f.jsonl; [ $rc -ne 0 ] && exit $rc
done
exit 0
