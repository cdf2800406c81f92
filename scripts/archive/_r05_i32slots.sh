#!/bin/bash
# Round 5 final: the int32x4 in-flight slot count (2 / 3), interleaved, four
# rounds, on the bench with the window's clock ramp.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r05i32slots; mkdir -p $O; : > $O/lines.jsonl
for r in 1 2 3 4; do
  for s in 2 3; do
    timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-host-path --no-extras --inflight $s > $O/b.json 2> $O/b.err || exit $?
    python -c "import json; d=json.loads(open('$O/b.json').read().splitlines()[-1]); print(json.dumps({'round': $r, 'slots': $s, 'ms': d['ms_per_step'], 'inflight_ms': d['frames_in_flight']['ms_per_step'], 'one_stream_ms': d['one_stream']['ms_per_step']}))" | tee -a $O/lines.jsonl
  done
done
