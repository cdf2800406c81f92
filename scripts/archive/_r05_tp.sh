#!/bin/bash
# Round 5: the C++ frame loop (rt_headless --throughput) and the trace_bin
# record-prefetch variant A/B.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r05tp; mkdir -p $O
timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py -k throughput > $O/tp_test.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 $O/tp_test.log; [ $rc -ne 0 ] && exit $rc
export LD_LIBRARY_PATH=opencl-ray-tracer_amd:${LD_LIBRARY_PATH:-}
for a in "--inflight 2" "--inflight 1" "--inflight 3 --format rgba8" "--inflight 1 --format rgba8"; do
  timeout -k 10 60 opencl-ray-tracer_amd/rt_headless --synthetic 256 64 6.4 --seed 3 --width 4096 --height 4096 --throughput 400 $a >> $O/headless.txt 2>&1
  rc=$?; [ $rc -ne 0 ] && { tail -3 $O/headless.txt; exit $rc; }
done
cat $O/headless.txt
V=opencl-ray-tracer_amd/variants
for f in i32x4 rgba8; do
  timeout -k 10 200 python scripts/bench_variants.py $V/librt_hip_base.so@trace_bin=1 $V/librt_hip_pf.so@trace_bin=1 --kernels --rounds 9 --format $f > $O/pf_$f.json 2>&1
  rc=$?; grep -v amdgpu $O/pf_$f.json; [ $rc -ne 0 ] && exit $rc
done
exit 0
