#!/bin/bash
# Round 4: first-call diagnosis + two/four-wave trace workgroups A/B
# (VERDICT r3 items 2 and 5).  Variants: scripts/variants.sh wg1/wg2/wg4.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r04b; mkdir -p $O
V=opencl-ray-tracer_amd/variants
timeout -k 10 120 python scripts/first_call.py > $O/first_call_a.json 2> $O/first_call_a.err || exit $?
timeout -k 10 120 python scripts/first_call.py --idle-ms 50 > $O/first_call_b.json 2> $O/first_call_b.err || exit $?
timeout -k 10 120 python scripts/first_call.py --warm-d2h 8000000 > $O/first_call_c.json 2> $O/first_call_c.err || exit $?
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
for f in rgba8 i32x4; do
  timeout -k 10 300 python scripts/bench_variants.py $V/librt_hip_wg1.so $V/librt_hip_wg2.so $V/librt_hip_wg4.so \
      --format $f --kernels --rounds 9 > $O/wg_$f.json 2> $O/wg_$f.err || exit $?
done
timeout -k 10 300 python scripts/bench_variants.py $V/librt_hip_wg1.so $V/librt_hip_wg2.so $V/librt_hip_wg4.so \
    --width 16384 --height 16384 --spheres 4096 --cubes 0 --seed 5 --kernels --rounds 5 --steps 5 \
    > $O/wg_c5d.json 2> $O/wg_c5d.err || exit $?
echo done
