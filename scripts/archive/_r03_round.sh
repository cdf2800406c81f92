#!/bin/bash
# Round 3: coarse classification rounds of 64 / 128 (32 does not fit the LDS alias) candidates.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
V=opencl-ray-tracer_amd/variants
L="$V/librt_hip_base.so $V/librt_hip_rd128.so"
timeout -k 10 200 python scripts/bench_variants.py $L --kernels --rounds 9 > gpurun_out/ab_round_c3.json 2>&1 || exit $?
timeout -k 10 200 python scripts/bench_variants.py $L --kernels --width 16384 --height 16384 --spheres 4096 --cubes 0 --seed 5 --k 25.6 --rounds 3 > gpurun_out/ab_round_c5d.json 2>&1 || exit $?
timeout -k 10 200 python scripts/bench_variants.py $L --kernels --width 8192 --height 8192 --spheres 192 --cubes 64 --seed 4 --rounds 3 > gpurun_out/ab_round_c4.json 2>&1 || exit $?
python scripts/show_ab.py gpurun_out/ab_round_*.json 2>/dev/null || true
