#!/bin/bash
# Frames in flight with the slots' traces chained (rt_set_trace_order) vs
# free, int32x4 and RGBA8.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out; export TMPDIR=/tmp
for fmt in i32x4 rgba8; do
  timeout -k 10 240 python scripts/inflight_cumask.py --format $fmt --settings 1:ffffffff 2:ffffffff,ffffffff "2:ffffffff,ffffffff|order" 3:ffffffff,ffffffff,ffffffff "3:ffffffff,ffffffff,ffffffff|order" "4:ffffffff,ffffffff,ffffffff,ffffffff|order" > gpurun_out/order_$fmt.txt 2>&1
  rc=$?; echo "== $fmt rc=$rc"; grep -v amdgpu.ids gpurun_out/order_$fmt.txt; [ $rc -ne 0 ] && exit $rc
done
echo done
