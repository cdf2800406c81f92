# A/B of RT_KTOUCH (trace3 touches a batch's record lines before the walk):
# configs 3, 4 and 5 dense, both formats.
# (The RT_KTOUCH code was measured and reverted, DESIGN.md §3 rejected table;
# rebuilding these variants needs it restored from git history.)
set -u
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
V=opencl-ray-tracer_amd/variants; O=gpurun_out/ab_ktouch.txt; : > $O
L="$V/librt_hip_base.so $V/librt_hip_kt1.so $V/librt_hip_kt2.so"
run() { echo "== $*" >> $O; timeout -k 10 300 python -u scripts/bench_variants.py $L --kernels "$@" >> $O 2>&1 || exit $?; }
run --format i32x4
run --format rgba8
run --width 8192 --height 8192 --spheres 192 --cubes 64 --seed 4 --rounds 5 --steps 10
run --width 16384 --height 16384 --spheres 4096 --cubes 0 --seed 5 --rounds 5 --steps 10
run --width 16384 --height 16384 --spheres 4096 --cubes 0 --seed 5 --rounds 5 --steps 10 --format rgba8
echo done
