#!/bin/bash
# Round 4: the sphere test on row pairs with packed fp32 (RT_PK_SPH) vs scalar.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r04j; mkdir -p $O
V=opencl-ray-tracer_amd/variants
L="$V/librt_hip_pk00.so $V/librt_hip_pk10.so $V/librt_hip_pk01.so $V/librt_hip_pk11.so"
for f in rgba8 i32x4; do
  timeout -k 10 300 python scripts/bench_variants.py $L --format $f --kernels --rounds 9 > $O/pk_c3_$f.json 2> $O/pk_c3_$f.err || exit $?
  timeout -k 10 300 python scripts/bench_variants.py $L --format $f --kernels --rounds 5 --steps 6 --width 16384 --height 16384 \
      --spheres 4096 --cubes 0 --seed 5 > $O/pk_c5_$f.json 2> $O/pk_c5_$f.err || exit $?
done
timeout -k 10 300 python scripts/bench_variants.py $L --kernels --rounds 7 --width 1920 --height 1080 \
      --spheres 16 --cubes 4 --seed 2 > $O/pk_c2.json 2> $O/pk_c2.err || exit $?
timeout -k 10 300 python scripts/bench_variants.py $L --kernels --rounds 7 --width 8192 --height 8192 \
      --spheres 192 --cubes 64 --seed 4 > $O/pk_c4.json 2> $O/pk_c4.err || exit $?
echo done
