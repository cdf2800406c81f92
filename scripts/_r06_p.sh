#!/bin/bash
# Round 6: the round-5 library (built from commit e961c9b's rt_device.hip /
# rt_trace.inc) against the round-6 final library in the bench's frame
# loops, interleaved: config 3 (both formats) and config 3 sparse.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r06p; mkdir -p $O
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
V=$PWD/opencl-ray-tracer_amd/variants
for round in 1 2 3; do
  for v in r05 r06; do
    RT_HIP_LIBRARY=$V/librt_hip_$v.so timeout -k 10 150 python bench.py --no-host-path --no-cpu-baseline \
        --steps 20 --warmup 5 --sustained 600 > $O/c3_${v}_$round.json 2> $O/c3_${v}_$round.err
    rc=$?; [ $rc -ne 0 ] && { tail -20 $O/c3_${v}_$round.err; exit $rc; }
    python -c "
import json; d=json.load(open('$O/c3_${v}_$round.json')); t=d['texture_rgba8']
print('c3 $v', $round, 'i32x4', d['ms_per_step'], d['frames_in_flight']['sustained']['ms_per_step'], d['roofline']['kernel_ms'], d['one_stream']['ms_per_step'], d['frame_check_ref'],
      'rgba8', t['ms_per_step'], t['frames_in_flight']['sustained']['ms_per_step'], t['roofline']['kernel_ms'], t['frame_check_ref'])"
  done
done
for round in 1 2; do
  for v in r05 r06; do
    RT_HIP_LIBRARY=$V/librt_hip_$v.so timeout -k 10 150 python bench.py --no-host-path --no-cpu-baseline --no-extras \
        --k 1 --steps 20 --warmup 5 --sustained 600 > $O/sparse_${v}_$round.json 2> $O/sparse_${v}_$round.err
    rc=$?; [ $rc -ne 0 ] && { tail -20 $O/sparse_${v}_$round.err; exit $rc; }
    python -c "
import json; d=json.load(open('$O/sparse_${v}_$round.json'))
print('sparse $v', $round, d['ms_per_step'], d['frames_in_flight']['ms_per_step'], d['frames_in_flight']['sustained']['ms_per_step'], d['roofline']['kernel_ms'], d['one_stream']['ms_per_step'])"
  done
done
echo done
