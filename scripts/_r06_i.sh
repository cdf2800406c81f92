#!/bin/bash
# Round 6: kernel-argument preloading into SGPRs (gfx950;
# -mllvm -amdgpu-kernarg-preload-count=16: a kernel's first 16 argument
# dwords arrive in user SGPRs, no scalar load in front of the first data
# load) against the shipped build: config 3 both formats, interleaved in one
# process, then the bench's frame loops, two interleaved rounds.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r06i; mkdir -p $O
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
V=opencl-ray-tracer_amd/variants
run() {  # name, args...
  local n=$1; shift
  timeout -k 10 300 python scripts/bench_variants.py $V/librt_hip_base.so $V/librt_hip_kp.so "$@" --kernels \
      > $O/$n.json 2> $O/$n.err
  rc=$?; echo "$n rc=$rc"; python -c "
import json; d=json.load(open('$O/$n.json')); print({k: (v['prep_us'], v['bin_us'], v['trace_us'], v['median_us']) for k, v in d.items()})"
  grep -h MISMATCH $O/$n.err; [ $rc -ne 0 ] && { tail -20 $O/$n.err; exit $rc; }
}
run i32x4 --rounds 9
run rgba8 --format rgba8 --rounds 9
run scene3 --scene 3 --rounds 9
for round in 1 2 3; do
  for v in base kp; do
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
