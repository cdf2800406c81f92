#!/bin/bash
# Round 6: the ballot-driven candidate walk in trace3_kernel (RT_WALK_BALLOT:
# the bin's list by vector loads, one keep ballot per 64 entries, only the
# kept entries visited) against the shipped walk (scalar batches of 8, every
# entry tested for its keep bit): RGBA8 / int32x4 config 3, config 5 dense,
# reference scene 3 at 640x480, interleaved in one process, frames bit-exact;
# then the frame loops.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r06g; mkdir -p $O
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
V=opencl-ray-tracer_amd/variants
run() {  # name, args...
  local n=$1; shift
  timeout -k 10 300 python scripts/bench_variants.py "$@" --kernels > $O/$n.json 2> $O/$n.err
  rc=$?; echo "$n rc=$rc"; python -c "
import json; d=json.load(open('$O/$n.json')); print({k: (v['trace_us'], v['bin_us'], v['median_us']) for k, v in d.items()})"
  grep -h MISMATCH $O/$n.err; [ $rc -ne 0 ] && { tail -20 $O/$n.err; exit $rc; }
}
run rgba8 $V/librt_hip_base.so $V/librt_hip_wb.so --format rgba8 --rounds 9
run i32x4_trace3 $V/librt_hip_base.so@trace_bin=2 $V/librt_hip_wb.so@trace_bin=2 --format i32x4 --rounds 7
run c5d $V/librt_hip_base.so $V/librt_hip_wb.so --width 16384 --height 16384 --spheres 4096 --cubes 0 --seed 5 --rounds 5 --steps 10
run c5d_rgba8 $V/librt_hip_base.so $V/librt_hip_wb.so --width 16384 --height 16384 --spheres 4096 --cubes 0 --seed 5 --rounds 5 --steps 10 --format rgba8
run c4 $V/librt_hip_base.so@trace_bin=2 $V/librt_hip_wb.so@trace_bin=2 --width 8192 --height 8192 --spheres 192 --cubes 64 --seed 4 --rounds 5 --steps 10
run scene3 $V/librt_hip_base.so $V/librt_hip_wb.so --scene 3 --rounds 9
for round in 1 2; do
  for v in base wb; do
    RT_HIP_LIBRARY=$PWD/$V/librt_hip_$v.so timeout -k 10 150 python bench.py --no-host-path --no-cpu-baseline \
        --steps 20 --warmup 5 --sustained 600 > $O/py_${v}_$round.json 2> $O/py_${v}_$round.err
    rc=$?; [ $rc -ne 0 ] && { tail -20 $O/py_${v}_$round.err; exit $rc; }
    python -c "
import json; d=json.load(open('$O/py_${v}_$round.json')); t=d['texture_rgba8']
print('$v', $round, 'i32x4', d['ms_per_step'], d['frames_in_flight']['sustained']['ms_per_step'], d['frame_check_ref'],
      'rgba8', t['ms_per_step'], t['frames_in_flight']['sustained']['ms_per_step'], t['roofline']['kernel_ms'], t['frame_check_ref'])"
  done
done
echo done
