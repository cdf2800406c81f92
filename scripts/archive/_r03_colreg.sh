#!/bin/bash
# Round 3: the hit colour kept in registers (RT_COL_REG=1) vs gathered after
# the walk (0): config 3 both formats, config 5 dense, config 4, the 8-rank band.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
V=opencl-ray-tracer_amd/variants
L="$V/librt_hip_col0.so $V/librt_hip_col1.so"
timeout -k 10 200 python scripts/bench_variants.py $L --kernels --rounds 9 > gpurun_out/ab_col_c3_i32.json 2>&1 || exit $?
timeout -k 10 200 python scripts/bench_variants.py $L --kernels --rounds 9 --format rgba8 > gpurun_out/ab_col_c3_rgba8.json 2>&1 || exit $?
timeout -k 10 200 python scripts/bench_variants.py $L --kernels --width 16384 --height 16384 --spheres 4096 --cubes 0 --seed 5 --k 25.6 --rounds 3 > gpurun_out/ab_col_c5d.json 2>&1 || exit $?
timeout -k 10 200 python scripts/bench_variants.py $L --kernels --width 8192 --height 8192 --spheres 192 --cubes 64 --seed 4 --rounds 3 > gpurun_out/ab_col_c4.json 2>&1 || exit $?
timeout -k 10 200 python scripts/bench_variants.py $L --kernels --ranks 8 > gpurun_out/ab_col_band8.json 2>&1 || exit $?
python scripts/show_ab.py gpurun_out/ab_col_*.json 2>/dev/null || true
echo done
