#!/bin/bash
# Round 3: the trace's sphere depth-cull test per lane + ballot (RT_LANE_CULL=1)
# vs the DPP wave maximum, interleaved in one process, frames bit-exact.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out; export TMPDIR=/tmp
V=opencl-ray-tracer_amd/variants
L="$V/librt_hip_base.so $V/librt_hip_lane.so"
timeout -k 10 150 python scripts/bench_variants.py $L --kernels --format rgba8 > gpurun_out/lane_c3_rgba8.json 2>&1 || { tail gpurun_out/lane_c3_rgba8.json; exit 1; }
timeout -k 10 150 python scripts/bench_variants.py $L --kernels > gpurun_out/lane_c3_i32.json 2>&1 || { tail gpurun_out/lane_c3_i32.json; exit 1; }
timeout -k 10 200 python scripts/bench_variants.py $L --kernels --width 16384 --height 16384 --spheres 4096 --cubes 0 --seed 5 --rounds 5 --steps 5 > gpurun_out/lane_c5d_i32.json 2>&1 || { tail gpurun_out/lane_c5d_i32.json; exit 1; }
timeout -k 10 200 python scripts/bench_variants.py $L --kernels --width 16384 --height 16384 --spheres 4096 --cubes 0 --seed 5 --rounds 5 --steps 5 --format rgba8 > gpurun_out/lane_c5d_rgba8.json 2>&1 || { tail gpurun_out/lane_c5d_rgba8.json; exit 1; }
for f in gpurun_out/lane_*.json; do echo "== $f"; grep -v amdgpu.ids $f; done
