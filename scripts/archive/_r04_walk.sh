#!/bin/bash
# Round 4: the candidate walk restructured (tests split into t + one update) vs before.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r04k; mkdir -p $O
V=opencl-ray-tracer_amd/variants
L="$V/librt_hip_old.so $V/librt_hip_new0.so $V/librt_hip_new1.so"
for f in rgba8 i32x4; do
  timeout -k 10 300 python scripts/bench_variants.py $L --format $f --kernels --rounds 9 > $O/walk_c3_$f.json 2> $O/walk_c3_$f.err || exit $?
  timeout -k 10 300 python scripts/bench_variants.py $L --format $f --kernels --rounds 5 --steps 6 --width 16384 --height 16384 \
      --spheres 4096 --cubes 0 --seed 5 > $O/walk_c5_$f.json 2> $O/walk_c5_$f.err || exit $?
done
timeout -k 10 300 python scripts/bench_variants.py $L --kernels --rounds 7 --width 1920 --height 1080 \
      --spheres 16 --cubes 4 --seed 2 > $O/walk_c2.json 2> $O/walk_c2.err || exit $?
timeout -k 10 300 python scripts/bench_variants.py $L --kernels --rounds 7 --width 8192 --height 8192 \
      --spheres 192 --cubes 64 --seed 4 > $O/walk_c4.json 2> $O/walk_c4.err || exit $?
echo done
