set -u
cd $GRAFT_REPO_ROOT
V=opencl-ray-tracer_amd/variants
L="$V/librt_hip_base.so $V/librt_hip_rot1.so $V/librt_hip_rot5.so"
echo "== config 3"
timeout -k 10 300 python scripts/bench_variants.py $L --rounds 15 --modes 0,1 2>&1 | grep -v amdgpu.ids || exit 3
echo "== config 5 dense"
timeout -k 10 300 python scripts/bench_variants.py $L --rounds 5 --steps 5 --width 16384 --height 16384 --spheres 4096 --cubes 0 2>&1 | grep -v amdgpu.ids || exit 3
echo "== config 3, rank 0 of 8"
timeout -k 10 300 python scripts/bench_variants.py $L --rounds 9 --ranks 8 2>&1 | grep -v amdgpu.ids || exit 3
echo "== timeline"
timeout -k 10 200 python scripts/timeline.py $V/librt_hip_tlrot.so 1 2>&1 | grep -v amdgpu.ids | tail -12
