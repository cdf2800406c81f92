#!/bin/bash
# Round 4: the triangle cull's band-size gate (RT_COARSE_CULL_TRI_BINS): the
# small-band sweep and scene 3 again, the GPU suite, the 4096-seed sweep.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export O=gpurun_out/r04t
bash scripts/_r04_gate3.sh || exit $?
L=opencl-ray-tracer_amd/librt_hip.so
for f in i32x4 rgba8; do
  timeout -k 10 200 python scripts/bench_variants.py $L --scene 3 --format $f --kernels --rounds 7 > $O/scene3_$f.json 2>$O/scene3_$f.err || exit $?
  cat $O/scene3_$f.json
done
timeout -k 10 900 python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu tests/ > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $O/pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
RT_SWEEP_SEEDS=4096 timeout -k 10 900 python -u -m pytest -q --timeout 120 --timeout-method thread \
    tests/test_gpu_configs.py -k randomized_parity_sweep > $O/parity_sweep_4096.log 2>&1
rc=$?; echo "sweep rc=$rc"; tail -2 $O/parity_sweep_4096.log
echo done
