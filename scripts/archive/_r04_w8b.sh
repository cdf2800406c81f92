#!/bin/bash
# Round 4: 8-wave coarse bins in bands of at most 256 bins (default now)
# against 4 waves; the GPU suite and the 4096-seed sweep.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r04y; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/ \
    -k "coarse_waves or split" > $O/pytest_w8.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 $O/pytest_w8.log; [ $rc -ne 0 ] && exit $rc
L=opencl-ray-tracer_amd/librt_hip.so
V="$L@coarse_waves=4 $L"
run() { name=$1; shift
  timeout -k 10 200 python scripts/bench_variants.py $V --kernels --rounds 7 "$@" > $O/$name.json 2> $O/$name.err
  rc=$?; echo "$name rc=$rc"; python3 -c "
import json;d=json.load(open('$O/$name.json'))
for k,v in d.items(): print(f\"  {k:45s} frame {v['median_us']:8.2f} bin {v['bin_us']:6.2f} trace {v['trace_us']:8.2f}\")"
  [ $rc -ne 0 ] && { tail -5 $O/$name.err; exit $rc; }; }
run scene3 --scene 3
run scene3_rgba8 --scene 3 --format rgba8
run 640x480_100 --width 640 --height 480 --spheres 100 --cubes 100 --seed 3
run 640x480_400 --width 640 --height 480 --spheres 400 --cubes 400 --seed 3
run 1280x720_100 --width 1280 --height 720 --spheres 100 --cubes 100 --seed 3
run 1280x720_400 --width 1280 --height 720 --spheres 400 --cubes 400 --seed 3
timeout -k 10 900 python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu tests/ > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $O/pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
RT_SWEEP_SEEDS=4096 timeout -k 10 900 python -u -m pytest -q --timeout 120 --timeout-method thread \
    tests/test_gpu_configs.py -k randomized_parity_sweep > $O/parity_sweep_4096.log 2>&1
rc=$?; echo "sweep rc=$rc"; tail -2 $O/parity_sweep_4096.log
echo done
