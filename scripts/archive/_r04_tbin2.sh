#!/bin/bash
# Round 4 experiment: the no-coarse trace (trace_bin) with frames in flight
# at config 3 (the headline's loop), both formats.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r04tb2; mkdir -p $O
for f in i32x4 rgba8; do
  timeout -k 10 300 python scripts/inflight.py --knob trace_bin --values 0,1 --slots 1,2,3 --format $f \
      > $O/inflight_$f.txt 2> $O/inflight_$f.err
  rc=$?; echo "inflight $f rc=$rc"; cat $O/inflight_$f.txt; [ $rc -ne 0 ] && { tail -5 $O/inflight_$f.err; exit $rc; }
done
echo done
