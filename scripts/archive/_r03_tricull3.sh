#!/bin/bash
# Round 3: RGBA8 frames (1-3 in flight) with the triangle cull gated as for
# int32x4 (g5) vs in every frame at per-tile thresholds 4 / 2 / 1 (config 3, config 4).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out; export TMPDIR=/tmp
V=opencl-ray-tracer_amd/variants
for rep in 1 2; do
 for v in g5 t4 t2 t1; do
  RT_HIP_LIBRARY=$PWD/$V/librt_hip_$v.so timeout -k 10 200 python scripts/inflight_cumask.py --format rgba8 --rounds 5 --settings 1:ffffffff 2:ffffffff,ffffffff 3:ffffffff,ffffffff,ffffffff > gpurun_out/tc3_c3_$v.txt 2>&1
  rc=$?; echo "== c3 $v rc=$rc"; grep -v amdgpu.ids gpurun_out/tc3_c3_$v.txt; [ $rc -ne 0 ] && exit $rc
 done
done
for v in g5 t4 t2 t1; do
  RT_HIP_LIBRARY=$PWD/$V/librt_hip_$v.so timeout -k 10 200 python scripts/inflight_cumask.py --format rgba8 --size 8192 --spheres 192 --cubes 64 --seed 4 --rounds 5 --steps 20 --settings 1:ffffffff 2:ffffffff,ffffffff 3:ffffffff,ffffffff,ffffffff > gpurun_out/tc3_c4_$v.txt 2>&1
  rc=$?; echo "== c4 $v rc=$rc"; grep -v amdgpu.ids gpurun_out/tc3_c4_$v.txt; [ $rc -ne 0 ] && exit $rc
done
echo done
