#!/bin/bash
# One GPU call: GPU parity tests, then interleaved A/B timing of two variant
# libraries (opencl-ray-tracer_amd/variants/librt_hip_<name>.so) on config 3,
# config 5 dense and rank 0's band of the 8-rank config-3 workload, then a
# rocprofv3 kernel-stats run of each.  Usage: scripts/_ab.sh A B (SKIP_TESTS=1
# skips the tests).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
V=opencl-ray-tracer_amd/variants
L="$V/librt_hip_$1.so $V/librt_hip_$2.so"
if [ "${SKIP_TESTS:-0}" != "1" ]; then
  timeout -k 10 400 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread \
      > gpurun_out/pytest_ab.log 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_ab.log
  [ $rc -ge 2 ] && exit $rc
fi
echo "== config 3"
timeout -k 10 300 python scripts/bench_variants.py $L --rounds 9 2>&1 | grep -v amdgpu.ids || exit 3
echo "== config 5 dense"
timeout -k 10 300 python scripts/bench_variants.py $L --rounds 5 --steps 5 --width 16384 \
    --height 16384 --spheres 4096 --cubes 0 2>&1 | grep -v amdgpu.ids || exit 3
echo "== config 3, rank 0 of 8"
timeout -k 10 300 python scripts/bench_variants.py $L --rounds 7 --ranks 8 2>&1 \
    | grep -v amdgpu.ids || exit 3
bash scripts/_prof_variants.sh "$1" "$2"
