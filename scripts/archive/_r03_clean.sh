#!/bin/bash
# Round 3: trace3 without the removed variant knobs (new) vs the previous
# source (old): frames bit-exact, timings; then the GPU parity suite.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
V=opencl-ray-tracer_amd/variants
L="$V/librt_hip_old.so $V/librt_hip_new.so"
timeout -k 10 200 python scripts/bench_variants.py $L --kernels --rounds 11 > gpurun_out/ab_clean_c3_i32.json 2>&1 || exit $?
timeout -k 10 200 python scripts/bench_variants.py $L --kernels --rounds 11 --format rgba8 > gpurun_out/ab_clean_c3_rgba8.json 2>&1 || exit $?
timeout -k 10 200 python scripts/bench_variants.py $L --kernels --width 16384 --height 16384 --spheres 4096 --cubes 0 --seed 5 --k 25.6 --rounds 3 > gpurun_out/ab_clean_c5d.json 2>&1 || exit $?
timeout -k 10 200 python scripts/bench_variants.py $L --kernels --width 8192 --height 8192 --spheres 192 --cubes 64 --seed 4 --rounds 3 > gpurun_out/ab_clean_c4.json 2>&1 || exit $?
python scripts/show_ab.py gpurun_out/ab_clean_*.json 2>/dev/null || true
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/pytest_clean.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_clean.log
