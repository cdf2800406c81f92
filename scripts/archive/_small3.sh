set -u
cd $GRAFT_REPO_ROOT
V=opencl-ray-tracer_amd/variants
L="$V/librt_hip_base.so $V/librt_hip_s8.so $V/librt_hip_s16.so"
echo "== 1920x1080 128+32 (512 prims)"
timeout -k 10 300 python scripts/bench_variants.py $L --rounds 9 --width 1920 --height 1080 --spheres 128 --cubes 32 2>&1 | grep -v amdgpu.ids || exit 3
echo "== 4096 128+32 (512 prims)"
timeout -k 10 300 python scripts/bench_variants.py $L --rounds 7 --width 4096 --height 4096 --spheres 128 --cubes 32 2>&1 | grep -v amdgpu.ids || exit 3
echo "== config 3"
timeout -k 10 300 python scripts/bench_variants.py $L --rounds 9 2>&1 | grep -v amdgpu.ids || exit 3
