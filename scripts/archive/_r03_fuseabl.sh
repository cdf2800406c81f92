#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
V=opencl-ray-tracer_amd/variants
L="$V/librt_hip_unfused.so $V/librt_hip_fused.so $V/librt_hip_prep_only.so $V/librt_hip_nodepth.so"
timeout -k 10 200 python scripts/bench_variants.py $L --kernels > gpurun_out/fuseabl_c3.json 2>&1 || exit $?
timeout -k 10 200 python scripts/bench_variants.py $L --kernels --width 8192 --height 8192 --spheres 192 --cubes 64 --seed 4 --k 12.8 --rounds 5 > gpurun_out/fuseabl_c4.json 2>&1 || exit $?
timeout -k 10 200 python scripts/inflight_cumask.py --settings "1:ffffffff" "2:ffffffff,ffffffff" "2:0000ffff,ffff0000" "2:00ffffff,ffffff00" "2:0fffffff,fffffff0" "3:ffffffff,ffffffff,ffffffff" > gpurun_out/inflight_cumask.txt 2>&1 || exit $?
timeout -k 10 200 python scripts/inflight_cumask.py --format rgba8 --settings "1:ffffffff" "2:ffffffff,ffffffff" "2:0000ffff,ffff0000" "2:00ffffff,ffffff00" > gpurun_out/inflight_cumask_rgba8.txt 2>&1 || exit $?
L2="opencl-ray-tracer_amd/variants/librt_hip_c2w8.so opencl-ray-tracer_amd/variants/librt_hip_c2w6.so opencl-ray-tracer_amd/variants/librt_hip_c2w5.so"
timeout -k 10 200 python scripts/bench_variants.py $L2 --kernels --width 1920 --height 1080 --spheres 16 --cubes 4 --seed 2 --k 3 > gpurun_out/c2w_c2.json 2>&1 || exit $?
timeout -k 10 200 python scripts/bench_variants.py $L2 --kernels --width 1920 --height 1080 --spheres 16 --cubes 4 --seed 2 --k 3 --format rgba8 > gpurun_out/c2w_c2_rgba8.json 2>&1 || exit $?
timeout -k 10 200 python scripts/bench_variants.py $L2 --kernels --width 512 --height 512 --spheres 4 --cubes 1 --seed 1 --k 0.8 > gpurun_out/c2w_c1.json 2>&1 || exit $?
