#!/bin/bash
# Round 6: the default bench line three times back to back on the final
# library (the overdraw verdict stored by the kernels): the K = 20 window's
# spread on one box beside the 600-frame window; then the Texture leg with 2
# slots instead of 3, twice (the copy every 8th frame is gone).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r06t; mkdir -p $O
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
for i in 1 2 3; do
  timeout -k 10 300 python bench.py > $O/bench_$i.json 2> $O/bench_$i.err
  rc=$?; echo "bench $i rc=$rc"; [ $rc -ne 0 ] && { tail -20 $O/bench_$i.err; exit $rc; }
  python -c "
import json; d=json.load(open('$O/bench_$i.json')); t=d['texture_rgba8']
print($i, d['value'], d['ms_per_step'], d['frames_in_flight']['sustained']['ms_per_step'], d['roofline']['kernel_ms'], d['roofline']['frame_frac'], d['frame_check_ref'],
      'rgba8', t['ms_per_step'], t['frames_in_flight']['sustained']['ms_per_step'], t['roofline']['frame_frac'], t['frame_check_ref'])"
done
for i in 1 2; do
  timeout -k 10 300 python bench.py --no-host-path --no-cpu-baseline --inflight-rgba8 2 > $O/bench_tex2_$i.json 2> $O/bench_tex2_$i.err
  rc=$?; echo "bench tex2 $i rc=$rc"; [ $rc -ne 0 ] && { tail -20 $O/bench_tex2_$i.err; exit $rc; }
  python -c "
import json; d=json.load(open('$O/bench_tex2_$i.json')); t=d['texture_rgba8']
print('tex2', $i, t['ms_per_step'], t['frames_in_flight']['sustained']['ms_per_step'], t['roofline']['frame_frac'], t['frame_check_ref'])"
done
echo done
