#!/bin/bash
# Round 6: kernel-argument preloading in the bench's frame loops (base vs
# kp), four interleaved rounds.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r06j; mkdir -p $O
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
V=opencl-ray-tracer_amd/variants
for round in 1 2 3 4; do
  for v in base kp; do
    RT_HIP_LIBRARY=$PWD/$V/librt_hip_$v.so timeout -k 10 150 python bench.py --no-host-path --no-cpu-baseline \
        --steps 20 --warmup 5 --sustained 600 > $O/py_${v}_$round.json 2> $O/py_${v}_$round.err
    rc=$?; [ $rc -ne 0 ] && { tail -20 $O/py_${v}_$round.err; exit $rc; }
    python -c "
import json; d=json.load(open('$O/py_${v}_$round.json')); t=d['texture_rgba8']
print('$v', $round, 'i32x4', d['ms_per_step'], d['frames_in_flight']['sustained']['ms_per_step'], d['roofline']['kernel_ms'], d['one_stream']['ms_per_step'], d['frame_check_ref'],
      'rgba8', t['ms_per_step'], t['frames_in_flight']['sustained']['ms_per_step'], t['roofline']['kernel_ms'], t['frame_check_ref'])"
  done
done
echo done
