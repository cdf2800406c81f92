set -e
V=opencl-ray-tracer_amd/variants
A="$V/librt_hip_${1:-nocull}.so $V/librt_hip_${2:-cull}.so"
echo "== config 3"; timeout -k 10 300 python scripts/bench_variants.py $A --rounds 7 2>&1 | grep -v amdgpu.ids
echo "== config 5 dense"; timeout -k 10 300 python scripts/bench_variants.py $A --rounds 5 --steps 5 --width 16384 --height 16384 --spheres 4096 --cubes 0 2>&1 | grep -v amdgpu.ids
echo "== config 5 sparse"; timeout -k 10 300 python scripts/bench_variants.py $A --rounds 5 --steps 5 --width 16384 --height 16384 --spheres 4096 --cubes 0 --k 1 2>&1 | grep -v amdgpu.ids
