set -u
cd $GRAFT_REPO_ROOT
V=opencl-ray-tracer_amd/variants
L="$V/librt_hip_base.so $V/librt_hip_s2.so $V/librt_hip_s4.so"
echo "== scene2-like 640x480 8+10"
timeout -k 10 300 python scripts/bench_variants.py $L --rounds 11 --width 640 --height 480 --spheres 8 --cubes 10 --k 1 2>&1 | grep -v amdgpu.ids || exit 3
echo "== 1920x1080 32+8"
timeout -k 10 300 python scripts/bench_variants.py $L --rounds 11 --width 1920 --height 1080 --spheres 32 --cubes 8 2>&1 | grep -v amdgpu.ids || exit 3
echo "== 1920x1080 64+16 (256 prims)"
timeout -k 10 300 python scripts/bench_variants.py $L --rounds 11 --width 1920 --height 1080 --spheres 64 --cubes 16 2>&1 | grep -v amdgpu.ids || exit 3
echo "== 4096 16+4"
timeout -k 10 300 python scripts/bench_variants.py $L --rounds 7 --width 4096 --height 4096 --spheres 64 --cubes 16 2>&1 | grep -v amdgpu.ids || exit 3
echo "== config 3"
timeout -k 10 300 python scripts/bench_variants.py $L --rounds 5 2>&1 | grep -v amdgpu.ids || exit 3
