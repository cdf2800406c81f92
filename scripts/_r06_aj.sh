#!/bin/bash
# Round 6: the int32x4 loop's slot count on the final library (the verdict
# copy every 8th frame is gone): 2 (default) against 3 slots, interleaved,
# four rounds, config 3.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r06aj; mkdir -p $O
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
for round in 1 2 3 4; do
  for n in 2 3; do
    timeout -k 10 200 python bench.py --no-host-path --no-cpu-baseline --no-extras --inflight $n > $O/i32_${n}_$round.json 2> $O/i32_${n}_$round.err
    rc=$?; [ $rc -ne 0 ] && { tail -20 $O/i32_${n}_$round.err; exit $rc; }
    python -c "
import json; d=json.load(open('$O/i32_${n}_$round.json'))
print('i32x4 slots $n', $round, 'window', d['ms_per_step'], 'sustained', d['frames_in_flight']['sustained']['ms_per_step'], d['frame_check_ref'])"
  done
done
echo done
