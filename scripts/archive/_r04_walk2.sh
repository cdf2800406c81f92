#!/bin/bash
# Round 4: the single-update walk in all three trace kernels ("all") vs in
# trace3 only ("cur"); then the GPU suite and the 4096-seed sweep on "all".
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r04l; mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
V=opencl-ray-tracer_amd/variants
L="$V/librt_hip_cur.so $V/librt_hip_all.so"
ab() { name=$1; shift
  timeout -k 10 300 python scripts/bench_variants.py $L --kernels --rounds 7 "$@" > $O/$name.json 2> $O/$name.err || exit $?; }
ab c2 --width 1920 --height 1080 --spheres 16 --cubes 4 --seed 2
ab c2_rgba8 --width 1920 --height 1080 --spheres 16 --cubes 4 --seed 2 --format rgba8
ab c1 --width 512 --height 512 --spheres 4 --cubes 1 --seed 1
ab small460 --width 4096 --height 1024 --spheres 100 --cubes 30 --seed 5 --k 6.4
ab small440 --width 1920 --height 1080 --spheres 200 --cubes 20 --seed 6 --k 3
ab c3_rgba8 --format rgba8
timeout -k 10 900 python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu tests/ > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $O/pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
RT_SWEEP_SEEDS=4096 timeout -k 10 900 python -u -m pytest -q --timeout 120 --timeout-method thread \
    tests/test_gpu_configs.py -k randomized_parity_sweep > $O/parity_sweep_4096.log 2>&1
rc=$?; echo "sweep rc=$rc"; tail -2 $O/parity_sweep_4096.log
echo done
