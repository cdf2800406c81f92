#!/bin/bash
# Round 5 checkpoint: the GPU suite, smoke + bench + rocprofv3 stats, and
# the RGBA8 no-coarse threshold with frames in flight.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r05c; mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu tests/ > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $O/pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
TAG=r05b SKIP_TESTS=1 bash scripts/gpu_check.sh || exit $?
for k in 1.0 4.5 6.4; do
  timeout -k 10 300 python scripts/inflight.py --format rgba8 --k $k --knob trace_path --values 0,1 --slots 1,3 >> $O/inflight_rgba8.txt 2>$O/inflight.err
  rc=$?; [ $rc -ne 0 ] && { tail -3 $O/inflight.err; exit $rc; }
done
cat $O/inflight_rgba8.txt
