#!/bin/bash
# Round 3: 8 rows per lane (16x32 wave tiles) at 8 / 6 / 5 / 4 waves per SIMD vs 4 rows.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
V=opencl-ray-tracer_amd/variants
L="$V/librt_hip_base.so $V/librt_hip_r8w8.so $V/librt_hip_r8w6.so $V/librt_hip_r8w5.so $V/librt_hip_r8w4.so"
timeout -k 10 200 python scripts/bench_variants.py $L --kernels --rounds 7 --format rgba8 > gpurun_out/ab_rows8_c3_rgba8.json 2>&1 || exit $?
timeout -k 10 200 python scripts/bench_variants.py $L --kernels --rounds 7 > gpurun_out/ab_rows8_c3_i32.json 2>&1 || exit $?
python scripts/show_ab.py gpurun_out/ab_rows8_*.json 2>/dev/null || true
