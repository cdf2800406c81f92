#!/bin/bash
# Round 5: the persistent coarse-path trace (trace3p_kernel) -- parity,
# then A/B against trace3_kernel (one stream and frames in flight).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r05p; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/ \
    -k "trace_persist" > $O/pytest.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 $O/pytest.log; [ $rc -ne 0 ] && exit $rc
run() { echo "== $*"; timeout -k 10 300 python scripts/ab_knob.py "$@" 2>&1 | grep -v amdgpu.ids | tee -a $O/ab.jsonl; r=${PIPESTATUS[0]}; [ $r -ne 0 ] && exit $r; return 0; }
run --knob trace_persist --values 0,6,4,3 --fixed trace_bin=2 --format i32x4 --configs c3,c3s,c4
run --knob trace_persist --values 0,6,4 --fixed trace_bin=2 --format rgba8 --configs c3,c4
timeout -k 10 300 python scripts/inflight.py --knob trace_persist --values 0,6 --fixed trace_bin=2 --slots 1,2,3 > $O/inflight.txt 2>$O/inflight.err
rc=$?; echo "inflight rc=$rc"; cat $O/inflight.txt; [ $rc -ne 0 ] && { tail -3 $O/inflight.err; exit $rc; }
timeout -k 10 300 python scripts/inflight.py --format rgba8 --knob trace_persist --values 0,6 --fixed trace_bin=2 --slots 1,3 > $O/inflight_rgba8.txt 2>>$O/inflight.err
rc=$?; echo "inflight rc=$rc"; cat $O/inflight_rgba8.txt; exit $rc
