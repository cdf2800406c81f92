#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
V=opencl-ray-tracer_amd/variants
L="$V/librt_hip_wg1.so $V/librt_hip_wg2.so $V/librt_hip_wg4.so"
timeout -k 10 200 python scripts/bench_variants.py $L --kernels --format rgba8 > gpurun_out/wg_c3_rgba8.json 2>&1 || exit $?
timeout -k 10 200 python scripts/bench_variants.py $L --kernels > gpurun_out/wg_c3_i32.json 2>&1 || exit $?
timeout -k 10 200 python scripts/bench_variants.py $L --kernels --width 16384 --height 16384 --spheres 4096 --cubes 0 --seed 5 --k 25.6 --rounds 3 > gpurun_out/wg_c5d.json 2>&1 || exit $?
timeout -k 10 200 python scripts/bench_variants.py $L --kernels --ranks 8 > gpurun_out/wg_band8.json 2>&1 || exit $?
