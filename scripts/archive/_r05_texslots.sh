#!/bin/bash
# Round 5 final: the Texture leg's slot count (2 / 3 / 4 frames in flight),
# interleaved, three rounds, on the bench with the window's clock ramp.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r05texslots; mkdir -p $O; : > $O/lines.jsonl
for r in 1 2 3; do
  for s in 2 3 4; do
    timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-host-path --inflight-rgba8 $s > $O/b.json 2> $O/b.err || exit $?
    python -c "import json; d=json.loads(open('$O/b.json').read().splitlines()[-1]); t=d['texture_rgba8']; print(json.dumps({'round': $r, 'slots': $s, 'tex_ms': t['ms_per_step'], 'i32_ms': d['ms_per_step']}))" | tee -a $O/lines.jsonl
  done
done
