#!/bin/bash
# Round 3: prep_kernel storing each triangle record as it is computed
# (RT_PREP_DIRECT=1) vs holding it in registers to the end (0).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out; export TMPDIR=/tmp
V=opencl-ray-tracer_amd/variants
L="$V/librt_hip_pd0.so $V/librt_hip_pd1.so"
run() { n=$1; shift; timeout -k 10 150 python scripts/bench_variants.py $L --kernels --rounds 9 "$@" > gpurun_out/pdirect_$n.json 2>&1 || { tail gpurun_out/pdirect_$n.json; exit 1; }; }
run c3
run c3_rgba8 --format rgba8
run c4 --width 8192 --height 8192 --spheres 192 --cubes 64 --seed 4 --steps 10
for f in gpurun_out/pdirect_*.json; do echo "== $f"; grep -v amdgpu.ids $f | tr -d '\n ' ; echo; done
