set -u
cd $GRAFT_REPO_ROOT
V=opencl-ray-tracer_amd/variants
L="$V/librt_hip_base.so $V/librt_hip_d4.so $V/librt_hip_d8.so"
for spec in "640 480 8 10 1" "1920 1080 32 8 3" "1920 1080 64 16 3" "1920 1080 100 30 3" "1920 1080 128 32 3" "4096 4096 128 32 6.4" "8192 8192 192 64 12.8"; do
  set -- $spec
  echo "== $1x$2 $3+$4"
  timeout -k 10 300 python scripts/bench_variants.py $L --rounds 9 --steps 10 --width $1 --height $2 --spheres $3 --cubes $4 --k $5 2>&1 | grep -v amdgpu.ids || exit 3
done
