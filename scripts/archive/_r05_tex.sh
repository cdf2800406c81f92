#!/bin/bash
# Round 5: why the bench's RGBA8 3-slot loop (39-40 us) trails
# scripts/inflight.py's (32.5 us) on the same frame: the bench with fewer
# earlier streams / other slot-stream kinds, then inflight.py.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r05tex; mkdir -p $O
B="--steps 20 --warmup 5 --no-cpu-baseline"
for v in "" "--no-host-path" "--slot-streams torch" "--slot-streams cumask" "--no-host-path --slot-streams torch"; do
  timeout -k 10 300 python bench.py $B $v > $O/b.json 2>$O/b.err
  rc=$?; [ $rc -ne 0 ] && { tail -3 $O/b.err; exit $rc; }
  python -c "
import json; d=json.loads(open('$O/b.json').read().splitlines()[-1]); t=d['texture_rgba8']
print('$v', 'i32x4', d['ms_per_step'], d['one_stream']['ms_per_step'], 'rgba8', t['ms_per_step'], t['one_stream']['ms_per_step'])" | tee -a $O/summary.txt
done
timeout -k 10 300 python scripts/inflight.py --format rgba8 --slots 1,2,3 | tee -a $O/summary.txt
