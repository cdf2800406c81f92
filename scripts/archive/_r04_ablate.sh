#!/bin/bash
# Round 4: trace-kernel ablations of the RGBA8 and int32x4 traces on the
# round-4 code (diagnostics build): 0 real, 1 stores only, 2 no per-pixel
# tests, 4 no colour gather.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r04g; mkdir -p $O
L=opencl-ray-tracer_amd/variants/librt_hip_diag.so
for f in rgba8 i32x4; do
  timeout -k 10 300 python scripts/bench_variants.py $L --format $f --kernels --rounds 7 --modes 0,1,2,4 \
      > $O/ablate_$f.json 2> $O/ablate_$f.err || exit $?
done
echo done
