#!/bin/bash
# Round 5: slot counts on CU-masked streams (int32x4 2/3, RGBA8 3/4/5).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r05sl; mkdir -p $O; : > $O/slots.jsonl
B="--steps 20 --warmup 5 --no-cpu-baseline --no-host-path"
for v in "--inflight 2 --inflight-rgba8 3" "--inflight 3 --inflight-rgba8 4" "--inflight 2 --inflight-rgba8 5" "--inflight 2 --inflight-rgba8 3"; do
  timeout -k 10 300 python bench.py $B $v > $O/b.json 2>$O/b.err
  rc=$?; [ $rc -ne 0 ] && { tail -3 $O/b.err; exit $rc; }
  python -c "
import json; d=json.loads(open('$O/b.json').read().splitlines()[-1]); t=d['texture_rgba8']
print(json.dumps({'args': '$v', 'i32x4': d['frames_in_flight']['ms_per_step'], 'i32x4_one': d['one_stream']['ms_per_step'], 'rgba8': t['frames_in_flight']['ms_per_step'], 'rgba8_one': t['one_stream']['ms_per_step']}))" | tee -a $O/slots.jsonl
done
