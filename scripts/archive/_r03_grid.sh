#!/bin/bash
# Round 3: trace3 2-D grid (no integer division) and trace occupancy variants.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
V=opencl-ray-tracer_amd/variants
L="$V/librt_hip_base.so $V/librt_hip_g2d.so $V/librt_hip_w6.so $V/librt_hip_w5.so"
timeout -k 10 200 python scripts/bench_variants.py $L --kernels > gpurun_out/ab_grid_c3_i32.json 2>&1 || exit $?
timeout -k 10 200 python scripts/bench_variants.py $L --kernels --format rgba8 > gpurun_out/ab_grid_c3_rgba8.json 2>&1 || exit $?
timeout -k 10 200 python scripts/bench_variants.py $L --kernels --width 16384 --height 16384 --spheres 4096 --cubes 0 --seed 5 --k 25.6 --rounds 3 > gpurun_out/ab_grid_c5d.json 2>&1 || exit $?
timeout -k 10 200 python scripts/bench_variants.py $L --kernels --ranks 8 > gpurun_out/ab_grid_band8.json 2>&1 || exit $?
