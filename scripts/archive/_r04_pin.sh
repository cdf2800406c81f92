#!/bin/bash
# Round 4: TriRec loaded in one round of scalar loads (RT_PIN_REC=1) vs two.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r04e; mkdir -p $O
V=opencl-ray-tracer_amd/variants
L="$V/librt_hip_pin0.so $V/librt_hip_pin1.so"
for f in rgba8 i32x4; do
  timeout -k 10 300 python scripts/bench_variants.py $L --format $f --kernels --rounds 9 > $O/pin_c3_$f.json 2> $O/pin_c3_$f.err || exit $?
  timeout -k 10 300 python scripts/bench_variants.py $L --format $f --kernels --rounds 7 --width 8192 --height 8192 \
      --spheres 192 --cubes 64 --seed 4 > $O/pin_c4_$f.json 2> $O/pin_c4_$f.err || exit $?
done
timeout -k 10 300 python scripts/bench_variants.py $L --kernels --rounds 7 --width 1920 --height 1080 \
      --spheres 16 --cubes 4 --seed 2 > $O/pin_c2.json 2> $O/pin_c2.err || exit $?
echo done
