#!/bin/bash
# Round 5: trace_tile_kernel (per-tile-strip masks, candidates walked from
# the mask words) -- parity, then A/B against the coarse path and
# trace_bin_kernel, one stream and frames in flight.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r05tile; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/ \
    -k "trace_tile or trace_bin_exact" > $O/pytest.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 $O/pytest.log; [ $rc -ne 0 ] && exit $rc
run() { echo "== $*"; timeout -k 10 300 python scripts/ab_knob.py "$@" 2>&1 | grep -v amdgpu.ids | tee -a $O/ab.jsonl; r=${PIPESTATUS[0]}; [ $r -ne 0 ] && exit $r; return 0; }
run --knob trace_path --values 0,1,2 --format i32x4 --configs c3,c3s,c3k15,c3k2,c2,p512
run --knob trace_path --values 0,1,2 --format rgba8 --configs c3,c3s
timeout -k 10 300 python scripts/inflight.py --knob trace_path --values 0,1,2 --slots 1,2,3 > $O/inflight.txt 2>$O/inflight.err
rc=$?; echo "inflight rc=$rc"; cat $O/inflight.txt; [ $rc -ne 0 ] && { tail -3 $O/inflight.err; exit $rc; }
timeout -k 10 300 python scripts/inflight.py --format rgba8 --knob trace_path --values 0,2 --slots 1,3 > $O/inflight_rgba8.txt 2>>$O/inflight.err
rc=$?; echo "inflight rc=$rc"; cat $O/inflight_rgba8.txt; exit $rc
