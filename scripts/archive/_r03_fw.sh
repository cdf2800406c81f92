#!/bin/bash
# Round 3: frame_small_kernel with 4 / 8 / 16 wave tiles per workgroup (configs 1, 2, both formats).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
V=opencl-ray-tracer_amd/variants
L="$V/librt_hip_fw4.so $V/librt_hip_fw8.so $V/librt_hip_fw16.so"
timeout -k 10 200 python scripts/bench_variants.py $L --kernels --rounds 9 --width 1920 --height 1080 --spheres 16 --cubes 4 --seed 2 > gpurun_out/ab_fw_c2.json 2>&1 || exit $?
timeout -k 10 200 python scripts/bench_variants.py $L --kernels --rounds 9 --width 1920 --height 1080 --spheres 16 --cubes 4 --seed 2 --format rgba8 > gpurun_out/ab_fw_c2_rgba8.json 2>&1 || exit $?
timeout -k 10 200 python scripts/bench_variants.py $L --kernels --rounds 9 --width 512 --height 512 --spheres 4 --cubes 1 --seed 1 > gpurun_out/ab_fw_c1.json 2>&1 || exit $?
python scripts/show_ab.py gpurun_out/ab_fw_*.json 2>/dev/null || true
