#!/bin/bash
# Round 4: frame stores as raw buffer stores (tile origin in the descriptor,
# 32-bit lane offset, the row step as the scalar offset) -- "bst" -- against
# the committed build ("base"), and "nz" (bst + no per-row t0 == 0 test
# where prep proves tmin > 0); then the GPU suite and the 4096-seed sweep.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r04o; mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
V=opencl-ray-tracer_amd/variants
L="$V/librt_hip_base.so $V/librt_hip_bst.so $V/librt_hip_nz.so"
ab() { name=$1; shift
  timeout -k 10 300 python scripts/bench_variants.py $L --kernels --rounds 7 "$@" > $O/$name.json 2> $O/$name.err
  rc=$?; echo "$name rc=$rc"; cat $O/$name.json; [ $rc -ne 0 ] && { tail -5 $O/$name.err; exit $rc; }; }
ab c3_rgba8 --format rgba8
ab c3_i32x4
ab c2 --width 1920 --height 1080 --spheres 16 --cubes 4 --seed 2
ab c4 --width 8192 --height 8192 --spheres 192 --cubes 64 --seed 4 --rounds 5
ab c5_i32x4 --width 16384 --height 16384 --spheres 4096 --cubes 0 --seed 5 --rounds 3 --steps 5
ab c5_rgba8 --width 16384 --height 16384 --spheres 4096 --cubes 0 --seed 5 --rounds 3 --steps 5 --format rgba8
ab scene3 --scene 3
ab scene3_rgba8 --scene 3 --format rgba8
ab small440 --width 1920 --height 1080 --spheres 200 --cubes 20 --seed 6 --k 3
timeout -k 10 900 python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu tests/ > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $O/pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
RT_SWEEP_SEEDS=4096 timeout -k 10 900 python -u -m pytest -q --timeout 120 --timeout-method thread \
    tests/test_gpu_configs.py -k randomized_parity_sweep > $O/parity_sweep_4096.log 2>&1
rc=$?; echo "sweep rc=$rc"; tail -2 $O/parity_sweep_4096.log
echo done
