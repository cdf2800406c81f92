#!/bin/bash
# Round 3: nontemporal frame stores per build and format: base (none), new
# (wide build, both formats), newn2 (also the 16x16 build's RGBA8 stores).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out; export TMPDIR=/tmp
V=opencl-ray-tracer_amd/variants
L="$V/librt_hip_base.so $V/librt_hip_new.so $V/librt_hip_newn2.so"
run() { n=$1; shift; timeout -k 10 200 python scripts/bench_variants.py $L --kernels "$@" > gpurun_out/nt2_$n.json 2>&1 || { tail gpurun_out/nt2_$n.json; exit 1; }; }
run c3_rgba8 --rounds 7 --format rgba8
run c4_rgba8 --width 8192 --height 8192 --spheres 192 --cubes 64 --seed 4 --steps 10 --rounds 7 --format rgba8
run c4 --width 8192 --height 8192 --spheres 192 --cubes 64 --seed 4 --steps 10 --rounds 7
run c5s --width 16384 --height 16384 --spheres 4096 --cubes 0 --seed 5 --k 1 --steps 5 --rounds 5
run c5d --width 16384 --height 16384 --spheres 4096 --cubes 0 --seed 5 --steps 5 --rounds 5
run c5d_rgba8 --width 16384 --height 16384 --spheres 4096 --cubes 0 --seed 5 --steps 5 --rounds 5 --format rgba8
for f in gpurun_out/nt2_*.json; do echo "== $f"; grep -v amdgpu.ids $f | tr -d '\n ' ; echo; done
