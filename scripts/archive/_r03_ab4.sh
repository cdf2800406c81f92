#!/bin/bash
# Round 3: A/B of four librt_hip variants (L1..L4 names) on config 3 (both
# formats), config 5 dense and the 8-rank band.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
V=opencl-ray-tracer_amd/variants; T=${TAG:-ab4}
L=""; for n in ${NAMES:-g2d xcd early both}; do L="$L $V/librt_hip_$n.so"; done
timeout -k 10 200 python scripts/bench_variants.py $L --kernels > gpurun_out/${T}_c3_i32.json 2>&1 || exit $?
timeout -k 10 200 python scripts/bench_variants.py $L --kernels --format rgba8 > gpurun_out/${T}_c3_rgba8.json 2>&1 || exit $?
timeout -k 10 200 python scripts/bench_variants.py $L --kernels --width 16384 --height 16384 --spheres 4096 --cubes 0 --seed 5 --k 25.6 --rounds 3 > gpurun_out/${T}_c5d.json 2>&1 || exit $?
timeout -k 10 200 python scripts/bench_variants.py $L --kernels --ranks 8 > gpurun_out/${T}_band8.json 2>&1 || exit $?
timeout -k 10 200 python scripts/bench_variants.py $L --kernels --width 8192 --height 8192 --spheres 192 --cubes 64 --seed 4 --k 12.8 --rounds 5 > gpurun_out/${T}_c4.json 2>&1 || exit $?
