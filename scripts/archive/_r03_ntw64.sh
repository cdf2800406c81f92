#!/bin/bash
# Round 3: the wide build's tile with nontemporal stores: 128x2 (kept) vs 64x4.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out; export TMPDIR=/tmp
V=opencl-ray-tracer_amd/variants
L="$V/librt_hip_w128.so $V/librt_hip_w64.so"
run() { n=$1; shift; timeout -k 10 200 python scripts/bench_variants.py $L --kernels "$@" > gpurun_out/ntw64_$n.json 2>&1 || { tail gpurun_out/ntw64_$n.json; exit 1; }; }
run c4 --width 8192 --height 8192 --spheres 192 --cubes 64 --seed 4 --steps 10 --rounds 7
run c5d --width 16384 --height 16384 --spheres 4096 --cubes 0 --seed 5 --steps 5 --rounds 5
run c5d_rgba8 --width 16384 --height 16384 --spheres 4096 --cubes 0 --seed 5 --steps 5 --rounds 5 --format rgba8
for f in gpurun_out/ntw64_*.json; do echo "== $f"; grep -v amdgpu.ids $f | tr -d '\n ' ; echo; done
