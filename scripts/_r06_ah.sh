#!/bin/bash
# Round 6: the Texture leg's slot count on the final library (the verdict
# copy every 8th frame is gone): 3 (default) against 4 slots, interleaved,
# four rounds, config 3.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r06ah; mkdir -p $O
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
for round in 1 2 3 4; do
  for n in 3 4; do
    timeout -k 10 200 python bench.py --no-host-path --no-cpu-baseline --inflight-rgba8 $n > $O/tex${n}_$round.json 2> $O/tex${n}_$round.err
    rc=$?; [ $rc -ne 0 ] && { tail -20 $O/tex${n}_$round.err; exit $rc; }
    python -c "
import json; d=json.load(open('$O/tex${n}_$round.json')); t=d['texture_rgba8']
print('slots $n', $round, 'window', t['ms_per_step'], 'sustained', t['frames_in_flight']['sustained']['ms_per_step'], t['frame_check_ref'], 'i32x4', d['ms_per_step'])"
  done
done
echo done
