#!/bin/bash
# Round 3: frame_small_kernel records as VGPR operands (broadcast LDS reads, RT_FUSED_VREC=1)
# vs moved to SGPRs by v_readfirstlane (0);
# and reference scene 2's size with 128 primitives (two chunks).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out; export TMPDIR=/tmp
V=opencl-ray-tracer_amd/variants
L="$V/librt_hip_vrec0.so $V/librt_hip_vrec1.so"
run() { n=$1; shift; timeout -k 10 120 python scripts/bench_variants.py $L --kernels --rounds 9 --steps 40 "$@" > gpurun_out/vrec_$n.json 2>&1 || { tail gpurun_out/vrec_$n.json; exit 1; }; }
run c1 --width 512 --height 512 --spheres 4 --cubes 1 --seed 1
run c2 --width 1920 --height 1080 --spheres 16 --cubes 4 --seed 2
run c2_rgba8 --width 1920 --height 1080 --spheres 16 --cubes 4 --seed 2 --format rgba8
run s128 --width 640 --height 480 --spheres 8 --cubes 10 --seed 1 --k 1.0
for f in gpurun_out/vrec_*.json; do echo "== $f"; grep -v amdgpu.ids $f | tr -d '\n ' ; echo; done
