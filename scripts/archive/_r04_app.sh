#!/bin/bash
# Reference scenes 1-3 at 640x480 (the app's own workload): per-kernel split.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out/r04n
L=opencl-ray-tracer_amd/librt_hip.so
for s in 1 2 3; do for f in i32x4 rgba8; do
  timeout -k 10 120 python scripts/bench_variants.py $L --scene $s --format $f --kernels --rounds 5 \
      > gpurun_out/r04n/scene${s}_$f.json 2>gpurun_out/r04n/scene${s}_$f.err
  rc=$?; echo "scene $s $f rc=$rc"; cat gpurun_out/r04n/scene${s}_$f.json
  [ $rc -ne 0 ] && { tail -5 gpurun_out/r04n/scene${s}_$f.err; exit $rc; }
done; done
echo done
