#!/bin/bash
# Round 6: candidate records addressed by a 32-bit byte offset (RT_REC_U32:
# a shorter scalar chain in front of each record's load) against the
# shipped build, interleaved in one process, then the bench's frame loops.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r06l; mkdir -p $O
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
V=opencl-ray-tracer_amd/variants
run() {  # name, args...
  local n=$1; shift
  timeout -k 10 300 python scripts/bench_variants.py "$@" --kernels > $O/$n.json 2> $O/$n.err
  rc=$?; echo "$n rc=$rc"; python -c "
import json; d=json.load(open('$O/$n.json')); print({k: (v['prep_us'], v['bin_us'], v['trace_us'], v['median_us']) for k, v in d.items()})"
  grep -h MISMATCH $O/$n.err; [ $rc -ne 0 ] && { tail -20 $O/$n.err; exit $rc; }
}
ALL="$V/librt_hip_base.so $V/librt_hip_ru.so"
run rgba8 $ALL --format rgba8 --rounds 9
run i32x4 $ALL --rounds 9
run i32x4_trace3 $V/librt_hip_base.so@trace_bin=2 $V/librt_hip_ru.so@trace_bin=2 --rounds 7
run scene3 $ALL --scene 3 --rounds 9
run c5d $ALL --width 16384 --height 16384 --spheres 4096 --cubes 0 --seed 5 --rounds 5 --steps 10
for round in 1 2 3; do
  for v in base ru; do
    RT_HIP_LIBRARY=$PWD/$V/librt_hip_$v.so timeout -k 10 150 python bench.py --no-host-path --no-cpu-baseline \
        --steps 20 --warmup 5 --sustained 600 > $O/py_${v}_$round.json 2> $O/py_${v}_$round.err
    rc=$?; [ $rc -ne 0 ] && { tail -20 $O/py_${v}_$round.err; exit $rc; }
    python -c "
import json; d=json.load(open('$O/py_${v}_$round.json')); t=d['texture_rgba8']
print('$v', $round, 'i32x4', d['ms_per_step'], d['frames_in_flight']['sustained']['ms_per_step'], d['roofline']['kernel_ms'], d['frame_check_ref'],
      'rgba8', t['ms_per_step'], t['frames_in_flight']['sustained']['ms_per_step'], t['roofline']['kernel_ms'], t['frame_check_ref'])"
  done
done
echo done
