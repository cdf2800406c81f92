#!/bin/bash
# Round 6: the final library's default bench line, three runs back to back
# (the K = 20 window's run-to-run spread).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r06n; mkdir -p $O
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
for i in 1 2 3; do
  timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_$i.json 2> $O/bench_$i.err
  rc=$?; echo "bench $i rc=$rc"; [ $rc -ne 0 ] && { tail -20 $O/bench_$i.err; exit $rc; }
  python -c "
import json; d=json.load(open('$O/bench_$i.json')); t=d['texture_rgba8']; f=d['frames_in_flight']
print($i, d['value'], d['ms_per_step'], f['sustained']['ms_per_step'], d['roofline']['kernel_ms'], d['roofline']['frac'], d['roofline']['frame_frac'], d['frame_check_ref'],
      '| tex', t['ms_per_step'], t['frames_in_flight']['sustained']['ms_per_step'], t['roofline']['frame_frac'], t['frame_check_ref'])"
done
echo done
