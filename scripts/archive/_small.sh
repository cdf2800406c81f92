set -u
cd $GRAFT_REPO_ROOT
timeout -k 10 500 python -u -m pytest tests -x -q -m gpu --timeout 200 --timeout-method thread > gpurun_out/pytest_small.log 2>&1; rc=$?; tail -4 gpurun_out/pytest_small.log; [ $rc -ne 0 ] && exit $rc
V=opencl-ray-tracer_amd/variants
L="$V/librt_hip_base.so $V/librt_hip_small.so"
echo "== config 2"
timeout -k 10 300 python scripts/bench_variants.py $L --rounds 11 --width 1920 --height 1080 --spheres 16 --cubes 4 2>&1 | grep -v amdgpu.ids || exit 3
echo "== config 1"
timeout -k 10 300 python scripts/bench_variants.py $L --rounds 11 --width 512 --height 512 --spheres 4 --cubes 1 2>&1 | grep -v amdgpu.ids || exit 3
echo "== config 3"
timeout -k 10 300 python scripts/bench_variants.py $L --rounds 7 2>&1 | grep -v amdgpu.ids || exit 3
