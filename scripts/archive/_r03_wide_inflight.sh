#!/bin/bash
# Round 3: frames in flight on the wide-tile build, 64x4 vs 128x2 tiles (config 4, config 5 sparse).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out; export TMPDIR=/tmp
V=opencl-ray-tracer_amd/variants
for v in w64 w128 w64 w128; do
  RT_HIP_LIBRARY=$PWD/$V/librt_hip_$v.so timeout -k 10 200 python scripts/inflight_cumask.py --size 8192 --spheres 192 --cubes 64 --seed 4 --rounds 5 --steps 20 --settings 1:ffffffff 2:ffffffff,ffffffff > gpurun_out/wide_inflight_c4_$v.txt 2>&1
  rc=$?; echo "== c4 $v rc=$rc"; grep -v amdgpu.ids gpurun_out/wide_inflight_c4_$v.txt; [ $rc -ne 0 ] && exit $rc
done
for v in w64 w128; do
  RT_HIP_LIBRARY=$PWD/$V/librt_hip_$v.so timeout -k 10 300 python scripts/inflight_cumask.py --size 16384 --spheres 4096 --cubes 0 --seed 5 --rounds 3 --steps 6 --settings 1:ffffffff 2:ffffffff,ffffffff > gpurun_out/wide_inflight_c5_$v.txt 2>&1
  rc=$?; echo "== c5d $v rc=$rc"; grep -v amdgpu.ids gpurun_out/wide_inflight_c5_$v.txt; [ $rc -ne 0 ] && exit $rc
done
