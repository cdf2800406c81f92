#!/bin/bash
# What prep and coarse cost a frame with frames in flight: diagnostic builds
# that skip prep (1), coarse (2) or both (3) after each context's first 16
# renders (the workspace keeps the lists, frames stay exact).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out; export TMPDIR=/tmp
V=opencl-ray-tracer_amd/variants
for fmt in i32x4 rgba8; do
  for lib in base skip1 skip2 skip3; do
    L=opencl-ray-tracer_amd/librt_hip.so; [ $lib != base ] && L=$V/librt_hip_$lib.so
    RT_HIP_LIBRARY=$PWD/$L timeout -k 10 240 python scripts/inflight_cumask.py --format $fmt --rounds 5 --settings 1:ffffffff 2:ffffffff,ffffffff 3:ffffffff,ffffffff,ffffffff > gpurun_out/skip_${fmt}_$lib.txt 2>&1
    rc=$?; echo "== $fmt $lib rc=$rc"; grep -v amdgpu.ids gpurun_out/skip_${fmt}_$lib.txt; [ $rc -ne 0 ] && exit $rc
  done
done
echo done
