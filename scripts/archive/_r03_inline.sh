#!/bin/bash
# Round 3: inline streams (trace4) vs id lists (trace3), interleaved A/B with
# frame checks, then the GPU suite on the new default.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
timeout -k 10 300 python scripts/ab_knob.py --knob inline_streams --values 0,1 --configs ${C_I32:-c3,c3s,c4,band8,c3x4,c5d,c5s} > gpurun_out/ab_inline_i32.jsonl 2>&1
rc=$?; echo "ab i32 rc=$rc"; [ $rc -ge 124 ] && exit $rc
timeout -k 10 300 python scripts/ab_knob.py --knob inline_streams --values 0,1 --format rgba8 --configs ${C_RGBA:-c3,c3s,c4,c5d} > gpurun_out/ab_inline_rgba8.jsonl 2>&1
rc=$?; echo "ab rgba8 rc=$rc"; [ $rc -ge 124 ] && exit $rc
if [ "${SKIP_TESTS:-0}" != 1 ]; then
timeout -k 10 500 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/pytest_inline.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/pytest_inline.log
fi
exit 0
