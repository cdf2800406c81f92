#!/bin/bash
# Round 5: frames-in-flight slot stream kinds on configs 3 (both formats), 4 and 5 dense.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r05s; mkdir -p $O; : > $O/streams.jsonl
B="--steps 20 --warmup 5 --no-cpu-baseline --no-host-path --no-extras"
for cfg in "" "--format rgba8 --inflight 3" "--width 8192 --height 8192 --spheres 192 --cubes 64 --seed 4" "--width 16384 --height 16384 --spheres 4096 --cubes 0 --seed 5"; do
  for kind in hip torch cumask; do
    timeout -k 10 300 python bench.py $B $cfg --slot-streams $kind > $O/b.json 2>$O/b.err
    rc=$?; [ $rc -ne 0 ] && { tail -3 $O/b.err; exit $rc; }
    python -c "
import json; d=json.loads(open('$O/b.json').read().splitlines()[-1]); f=d['frames_in_flight'] or {}
r={'cfg': '$cfg', 'kind': '$kind', 'one_stream': d['one_stream']['ms_per_step'], 'inflight': f.get('ms_per_step'), 'slots': f.get('frames_in_flight'), 'check': f.get('frame_check')}
print(json.dumps(r))" | tee -a $O/streams.jsonl
  done
done
