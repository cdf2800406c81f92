set -u
cd $GRAFT_REPO_ROOT
V=opencl-ray-tracer_amd/variants
L="$V/librt_hip_base.so $V/librt_hip_p1.so $V/librt_hip_p3.so"
echo "== config 3"
timeout -k 10 300 python scripts/bench_variants.py $L --rounds 11 2>&1 | grep -v amdgpu.ids || exit 3
echo "== config 5 dense"
timeout -k 10 300 python scripts/bench_variants.py $L --rounds 5 --steps 5 --width 16384 --height 16384 --spheres 4096 --cubes 0 2>&1 | grep -v amdgpu.ids || exit 3
echo "== config 3, rank 0 of 8"
timeout -k 10 300 python scripts/bench_variants.py $L --rounds 7 --ranks 8 2>&1 | grep -v amdgpu.ids || exit 3
