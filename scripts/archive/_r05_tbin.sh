#!/bin/bash
# Round 5: the no-coarse path (trace_bin_kernel) with the verdict word's
# lifetime fixed: its tests first, then frames in flight with the knob at
# auto / never, then the full GPU suite.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r05tb; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/ \
    -k "trace_bin or last_kernel or fresh_context or first_render" > $O/pytest_tbin.log 2>&1
rc=$?; echo "tbin tests rc=$rc"; tail -15 $O/pytest_tbin.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python scripts/inflight.py --knob trace_bin --values 0,2 --slots 1,2,3 > $O/inflight.txt 2>$O/inflight.err
rc=$?; echo "inflight rc=$rc"; cat $O/inflight.txt; [ $rc -ne 0 ] && { tail -5 $O/inflight.err; exit $rc; }
timeout -k 10 900 python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu tests/ > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $O/pytest_gpu.log; exit $rc
