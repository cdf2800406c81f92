#!/bin/bash
# Round 5 final: the clock ramp's length before the timed windows (50 / 200
# / 500 ms of untimed load), interleaved, three rounds.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r05ramp; mkdir -p $O; : > $O/lines.jsonl
for r in 1 2 3; do
  for m in 50 200 500; do
    timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-host-path --warmup-ms $m > $O/b.json 2> $O/b.err || exit $?
    python -c "import json; d=json.loads(open('$O/b.json').read().splitlines()[-1]); print(json.dumps({'round': $r, 'ramp_ms': $m, 'ms': d['ms_per_step'], 'one_stream_ms': d['one_stream']['ms_per_step'], 'tex_ms': d['texture_rgba8']['ms_per_step']}))" | tee -a $O/lines.jsonl
  done
done
