#!/bin/bash
# Round 4: the automatic no-coarse path (trace_bin_kernel below overdraw 6,
# int32x4, frames above 4096 wave tiles): its tests, the GPU suite, the
# 4096-seed sweep, then the round-end check (smoke, bench, rocprof).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r04tb4; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/ \
    -k "trace_bin or last_kernel" > $O/pytest_tbin.log 2>&1
rc=$?; echo "tbin tests rc=$rc"; tail -3 $O/pytest_tbin.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python scripts/inflight.py --knob trace_bin --values 0,2 --slots 1,2 > $O/inflight.txt 2>$O/inflight.err
rc=$?; echo "inflight rc=$rc"; cat $O/inflight.txt; [ $rc -ne 0 ] && { tail -5 $O/inflight.err; exit $rc; }
timeout -k 10 900 python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu tests/ > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $O/pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
RT_SWEEP_SEEDS=4096 timeout -k 10 900 python -u -m pytest -q --timeout 120 --timeout-method thread \
    tests/test_gpu_configs.py -k randomized_parity_sweep > $O/parity_sweep_4096.log 2>&1
rc=$?; echo "sweep rc=$rc"; tail -2 $O/parity_sweep_4096.log; [ $rc -ne 0 ] && exit $rc
TAG=r04tb SKIP_TESTS=1 bash scripts/gpu_check.sh
