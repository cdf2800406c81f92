#!/bin/bash
# Round 4: waves per coarse bin with frames in flight at config 3 (the
# headline's loop), both formats.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r04cwif; mkdir -p $O
for f in i32x4 rgba8; do
  timeout -k 10 300 python scripts/inflight.py --knob coarse_waves --values 0,2,4 --slots 1,2,3 --format $f \
      > $O/inflight_$f.txt 2> $O/inflight_$f.err
  rc=$?; echo "inflight $f rc=$rc"; cat $O/inflight_$f.txt; [ $rc -ne 0 ] && { tail -5 $O/inflight_$f.err; exit $rc; }
done
echo done
