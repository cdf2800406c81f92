#!/bin/bash
# Round 6: the ballot walk in trace3_split_kernel (small frames: 2 / 4 waves
# per tile) against the batch walk, on the small frames that take it, both
# formats, interleaved in one process; then the GPU suite and the 4096-seed
# sweep on the library with it on (the default).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r06h; mkdir -p $O
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
V=opencl-ray-tracer_amd/variants
run() {  # name, args...
  local n=$1; shift
  timeout -k 10 300 python scripts/bench_variants.py $V/librt_hip_base.so $V/librt_hip_sp.so "$@" --kernels --rounds 9 \
      > $O/$n.json 2> $O/$n.err
  rc=$?; echo "$n rc=$rc"; python -c "
import json; d=json.load(open('$O/$n.json')); print({k: (v['trace_us'], v['bin_us'], v['median_us']) for k, v in d.items()})"
  grep -h MISMATCH $O/$n.err; [ $rc -ne 0 ] && { tail -20 $O/$n.err; exit $rc; }
}
run scene3 --scene 3
run scene3_rgba8 --scene 3 --format rgba8
run s640_od --width 640 --height 480 --spheres 400 --cubes 40 --k 1.5
run s640_od_rgba8 --width 640 --height 480 --spheres 400 --cubes 40 --k 1.5 --format rgba8
run s720 --width 1280 --height 720 --spheres 256 --cubes 64 --k 2
run s720_rgba8 --width 1280 --height 720 --spheres 256 --cubes 64 --k 2 --format rgba8
run s1080 --width 1920 --height 1080 --spheres 256 --cubes 64 --k 3
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 240 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $O/pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
RT_SWEEP_SEEDS=4096 timeout -k 10 600 python -u -m pytest -q --timeout 120 --timeout-method thread \
    tests/test_gpu_configs.py -k randomized_parity_sweep > $O/parity_sweep_4096.log 2>&1
rc=$?; echo "sweep rc=$rc"; tail -2 $O/parity_sweep_4096.log
echo done
