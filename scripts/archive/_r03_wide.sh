#!/bin/bash
# Round 3: the wide-tile build (frames >= 512 MiB) at 64x4 / 128x2 / 256x1 tiles (32x8 measured first, slower).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
V=opencl-ray-tracer_amd/variants
L="$V/librt_hip_base.so $V/librt_hip_w128.so $V/librt_hip_w256.so"
timeout -k 10 200 python scripts/bench_variants.py $L --kernels --width 8192 --height 8192 --spheres 192 --cubes 64 --seed 4 --rounds 5 > gpurun_out/ab_wide2_c4.json 2>&1 || exit $?
timeout -k 10 200 python scripts/bench_variants.py $L --kernels --width 8192 --height 8192 --spheres 192 --cubes 64 --seed 4 --rounds 5 --format rgba8 > gpurun_out/ab_wide2_c4_rgba8.json 2>&1 || exit $?
timeout -k 10 300 python scripts/bench_variants.py $L --kernels --width 16384 --height 16384 --spheres 4096 --cubes 0 --seed 5 --k 25.6 --rounds 3 > gpurun_out/ab_wide2_c5d.json 2>&1 || exit $?
timeout -k 10 300 python scripts/bench_variants.py $L --kernels --width 16384 --height 16384 --spheres 4096 --cubes 0 --seed 5 --k 1 --rounds 3 > gpurun_out/ab_wide2_c5s.json 2>&1 || exit $?
python scripts/show_ab.py gpurun_out/ab_wide2_*.json 2>/dev/null || true
