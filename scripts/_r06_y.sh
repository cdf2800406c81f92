#!/bin/bash
# Round 6: the host's wait in the timed regions.  The bench with
# hipDeviceScheduleSpin (--sync-wait spin, the new default) against HIP's
# default wait, interleaved, three rounds (--sync-wait existed in bench.py
# while this was measured; not kept); then scripts/window_fill.py (the
# K-window's fixed cost and per-frame completion times) under spin.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r06y; mkdir -p $O
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
for round in 1 2 3; do
  for m in default spin; do
    timeout -k 10 300 python bench.py --no-cpu-baseline --sync-wait $m > $O/bench_${m}_$round.json 2> $O/bench_${m}_$round.err
    rc=$?; [ $rc -ne 0 ] && { tail -20 $O/bench_${m}_$round.err; exit $rc; }
    python -c "
import json; d=json.load(open('$O/bench_${m}_$round.json')); t=d['texture_rgba8']; a=d['host_path']['app']
print('$m', $round, d['sync_wait'], d['value'], d['ms_per_step'], d['frames_in_flight']['sustained']['ms_per_step'], d['one_stream']['ms_per_step'], d['frame_check_ref'],
      'rgba8', t['ms_per_step'], t['frames_in_flight']['sustained']['ms_per_step'], t['frame_check_ref'], 'app', json.dumps(a)[:300])"
  done
done
timeout -k 10 240 python scripts/window_fill.py i32x4 > $O/wf_i32x4.json 2> $O/wf_i32x4.err
rc=$?; [ $rc -ne 0 ] && { tail -20 $O/wf_i32x4.err; exit $rc; }
timeout -k 10 240 python scripts/window_fill.py rgba8 > $O/wf_rgba8.json 2> $O/wf_rgba8.err
rc=$?; [ $rc -ne 0 ] && { tail -20 $O/wf_rgba8.err; exit $rc; }
echo done
