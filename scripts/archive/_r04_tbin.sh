#!/bin/bash
# Round 4 experiment: binned frames without the coarse kernel
# (trace_bin_kernel) against prep -> coarse -> trace: parity tests first,
# then interleaved A/B, then the GPU suite and the sweep.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r04tb; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/ \
    -k "trace_bin" > $O/pytest_tbin.log 2>&1
rc=$?; echo "tbin tests rc=$rc"; tail -3 $O/pytest_tbin.log; [ $rc -ne 0 ] && exit $rc
L=opencl-ray-tracer_amd/librt_hip.so
V="$L $L@trace_bin=1"
run() { name=$1; shift
  timeout -k 10 300 python scripts/bench_variants.py $V --kernels --rounds 7 "$@" > $O/$name.json 2> $O/$name.err
  rc=$?; echo "$name rc=$rc"; python3 -c "
import json;d=json.load(open('$O/$name.json'))
for k,v in d.items(): print(f\"  {k:32s} frame {v['median_us']:8.2f} prep {v['prep_us']:6.2f} bin {v['bin_us']:6.2f} trace {v['trace_us']:8.2f}\")"
  [ $rc -ne 0 ] && { tail -5 $O/$name.err; exit $rc; }; }
run c3
run c3_rgba8 --format rgba8
run c4 --width 8192 --height 8192 --spheres 192 --cubes 64 --seed 4 --rounds 5
run c4_rgba8 --width 8192 --height 8192 --spheres 192 --cubes 64 --seed 4 --rounds 5 --format rgba8
run c3_sparse --k 1
run 2048_320 --width 2048 --height 2048 --spheres 256 --cubes 64 --seed 3
timeout -k 10 900 python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu tests/ > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $O/pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
RT_SWEEP_SEEDS=1024 timeout -k 10 600 python -u -m pytest -q --timeout 120 --timeout-method thread \
    tests/test_gpu_configs.py -k randomized_parity_sweep > $O/parity_sweep_1024.log 2>&1
rc=$?; echo "sweep rc=$rc"; tail -2 $O/parity_sweep_1024.log
echo done
