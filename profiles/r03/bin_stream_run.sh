#!/bin/bash
# Binning stream (rt_set_bin_stream) on one GPU: its parity tests, then
# frames in flight with and without a shared, CU-masked binning stream
# (scripts/inflight_cumask.py), int32x4 and RGBA8.  Stops at the first
# failing step.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m pytest tests -x -q -m gpu -k "bin_stream or golden_frame" --timeout 120 --timeout-method thread > gpurun_out/binstream_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/binstream_tests.log; [ $rc -ne 0 ] && exit $rc
S=(${SETTINGS:-"1:ffffffff" "2:ffffffff,ffffffff" "2:ffffffff,ffffffff|bin=ffffffff" "2:ffffffff,ffffffff|bin=01010101" "2:ffffffff,ffffffff|bin=11111111" "2:fefefefe,fefefefe|bin=01010101" "2:eeeeeeee,eeeeeeee|bin=11111111" "2:ffffffff,ffffffff|bin=00010001"})
for fmt in i32x4 rgba8; do
  timeout -k 10 300 python scripts/inflight_cumask.py --format $fmt --settings "${S[@]}" > gpurun_out/binstream_$fmt.txt 2>&1
  rc=$?; echo "$fmt rc=$rc"; cat gpurun_out/binstream_$fmt.txt; [ $rc -ne 0 ] && exit $rc
done
echo done
