#!/bin/bash
# Round 6: the overdraw-verdict copy period (RT_VERDICT_EVERY: one 4-byte
# D2H copy per 8 / 2 / 1 binned launches) in the bench's frame loops,
# three interleaved rounds, frames checked against the fixture.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r06e; mkdir -p $O
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
V=$PWD/opencl-ray-tracer_amd/variants
timeout -k 10 300 python scripts/bench_variants.py $V/librt_hip_base.so $V/librt_hip_ve2.so $V/librt_hip_ve1.so \
    --kernels --rounds 9 > $O/ab_i32x4.json 2> $O/ab_i32x4.err
rc=$?; echo "ab rc=$rc"; cat $O/ab_i32x4.json; [ $rc -ne 0 ] && { tail -20 $O/ab_i32x4.err; exit $rc; }
for round in 1 2 3; do
  for v in base ve2 ve1; do
    RT_HIP_LIBRARY=$V/librt_hip_$v.so timeout -k 10 150 python bench.py --no-host-path --no-cpu-baseline \
        --steps 20 --warmup 5 --sustained 600 > $O/py_${v}_$round.json 2> $O/py_${v}_$round.err
    rc=$?; [ $rc -ne 0 ] && { tail -20 $O/py_${v}_$round.err; exit $rc; }
    python -c "
import json; d=json.load(open('$O/py_${v}_$round.json')); t=d['texture_rgba8']
print('$v', $round, 'i32x4', d['ms_per_step'], d['frames_in_flight']['sustained']['ms_per_step'], d['frame_check_ref'],
      'rgba8', t['ms_per_step'], t['frames_in_flight']['sustained']['ms_per_step'], t['frame_check_ref'])"
  done
done
echo done1
# the rocprofv3 evidence of the bench command the profiler runs with: the
# default command with --sustained 0 (the 600-frame windows' overlapping
# launches would pull the kernel average up)
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/$O/prof" -o run --output-format csv -- \
    python "$GRAFT_REPO_ROOT/bench.py" --steps 20 --warmup 5 --sustained 0 > "$GRAFT_REPO_ROOT/$O/prof_bench.json" 2> "$GRAFT_REPO_ROOT/$O/prof_bench.err"
rc=$?; echo "rocprof rc=$rc"; [ $rc -ne 0 ] && { tail -20 "$GRAFT_REPO_ROOT/$O/prof_bench.err"; exit $rc; }
cd "$GRAFT_REPO_ROOT"
python scripts/rocprof_launches.py $O/prof/run_kernel_trace.csv trace_bin_kernel
grep '^{' $O/prof_bench.json | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['roofline'])"
echo done2
