#!/bin/bash
# Round 5: trace_bin_kernel's per-tile depth cull -- parity, then A/B
# against the coarse path (RGBA8) and cull on/off (both formats).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r05tc; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/ \
    -k "trace_bin or last_kernel" > $O/pytest_tbin.log 2>&1
rc=$?; echo "tbin tests rc=$rc"; tail -3 $O/pytest_tbin.log; [ $rc -ne 0 ] && exit $rc
run() { echo "== $*"; timeout -k 10 300 python scripts/ab_knob.py "$@" 2>&1 | tee -a $O/ab.jsonl; r=${PIPESTATUS[0]}; [ $r -ne 0 ] && exit $r; return 0; }
run --knob trace_bin --values 2,1 --format rgba8 --configs c3,c3s,c3k15,c3k2,c3k4
run --knob trace_bin_cull --values 0,1 --fixed trace_bin=1 --format rgba8 --configs c3,c3k2,c3k4
run --knob trace_bin_cull --values 0,1 --fixed trace_bin=1 --format i32x4 --configs c3,c3s,c3k15,c3k2,c3k4
run --knob trace_bin --values 2,1 --fixed trace_bin_cull=1 --format i32x4 --configs c3k15,c3k2,c3k4
timeout -k 10 300 python scripts/inflight.py --format rgba8 --knob trace_bin --values 2,1 --slots 1,2,3 > $O/inflight_rgba8.txt 2>$O/inflight.err
rc=$?; echo "inflight rc=$rc"; cat $O/inflight_rgba8.txt; exit $rc
