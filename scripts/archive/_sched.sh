# A/B of LLVM AMDGPU scheduler strategies (whole library rebuilt with
# -mllvm -amdgpu-sched-strategy=...), configs 3 and 5 dense, both formats.
set -u
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
V=opencl-ray-tracer_amd/variants; O=gpurun_out/ab_sched.txt; : > $O
L="$V/librt_hip_base.so $V/librt_hip_mmc.so $V/librt_hip_milp.so $V/librt_hip_itilp.so"
run() { echo "== $*" >> $O; timeout -k 10 300 python -u scripts/bench_variants.py $L --kernels "$@" >> $O 2>&1 || exit $?; }
run --format i32x4
run --format rgba8
run --width 16384 --height 16384 --spheres 4096 --cubes 0 --seed 5 --rounds 5 --steps 10
run --width 16384 --height 16384 --spheres 4096 --cubes 0 --seed 5 --rounds 5 --steps 10 --format rgba8
echo done
