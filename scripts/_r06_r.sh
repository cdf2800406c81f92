#!/bin/bash
# Round 6: the overdraw verdict written by the kernels straight into the
# host's mapped word (RT_VERDICT_DIRECT) against the copy every 8th binned
# launch: the path choice's lag (scripts/verdict_lag.py), the automatic-choice
# and config-3 tests on the direct build, and the bench's frame loops
# interleaved (config 3, both formats).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r06r; mkdir -p $O
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
V=$PWD/opencl-ray-tracer_amd/variants
for v in vcopy vdirect; do
  RT_HIP_LIBRARY=$V/librt_hip_$v.so timeout -k 10 120 python scripts/verdict_lag.py > $O/lag_$v.json 2> $O/lag_$v.err
  rc=$?; [ $rc -ne 0 ] && { tail -20 $O/lag_$v.err; exit $rc; }
  python -c "
import json; d=json.load(open('$O/lag_$v.json')); print('$v', ' '.join(n[0][0]+':'+k.replace('_kernel','') for n, k in [((a,), b) for a, b in d['frames']]))"
done
RT_HIP_LIBRARY=$V/librt_hip_vdirect.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread \
    -k "automatic_choice or config3_full_frame or trace_bin or last_kernel" -m gpu > $O/pytest_vdirect.log 2>&1
rc=$?; tail -3 $O/pytest_vdirect.log; [ $rc -ne 0 ] && exit $rc
for round in 1 2 3; do
  for v in vcopy vdirect; do
    RT_HIP_LIBRARY=$V/librt_hip_$v.so timeout -k 10 150 python bench.py --no-host-path --no-cpu-baseline \
        --steps 20 --warmup 5 --sustained 600 > $O/c3_${v}_$round.json 2> $O/c3_${v}_$round.err
    rc=$?; [ $rc -ne 0 ] && { tail -20 $O/c3_${v}_$round.err; exit $rc; }
    python -c "
import json; d=json.load(open('$O/c3_${v}_$round.json')); t=d['texture_rgba8']
print('c3 $v', $round, 'i32x4', d['ms_per_step'], d['frames_in_flight']['sustained']['ms_per_step'], d['roofline']['kernel_ms'], d['one_stream']['ms_per_step'], d['frame_check_ref'],
      'rgba8', t['ms_per_step'], t['frames_in_flight']['sustained']['ms_per_step'], t['roofline']['kernel_ms'], t['frame_check_ref'])"
  done
done
echo done
