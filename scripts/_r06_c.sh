#!/bin/bash
# Round 6: the 8-rows-per-lane RGBA8 trace in the frame loop -- bench.py's
# Texture leg (Python) at 2/3/4 slots and the C++ loop (rt_headless
# --throughput) at 2/3/4 slots, base against r8g2, three interleaved rounds.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r06c; mkdir -p $O
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
V=$PWD/opencl-ray-tracer_amd/variants
for v in base r8g2; do mkdir -p $O/lib_$v && cp $V/librt_hip_$v.so $O/lib_$v/librt_hip.so; done
for round in 1 2 3; do
  for v in base r8g2; do
    for s in 3 4; do
      RT_HIP_LIBRARY=$V/librt_hip_$v.so timeout -k 10 120 python bench.py --format rgba8 --no-extras --no-host-path \
          --no-cpu-baseline --inflight $s --steps 20 --warmup 5 --sustained 600 > $O/py_${v}_${s}_$round.json 2> $O/py_${v}_${s}_$round.err
      rc=$?; [ $rc -ne 0 ] && { tail -20 $O/py_${v}_${s}_$round.err; exit $rc; }
      python -c "import json; d=json.load(open('$O/py_${v}_${s}_$round.json')); f=d['frames_in_flight']; print('py $v', $s, $round, d['ms_per_step'], f['ms_per_step'], f['sustained']['ms_per_step'], d['frame_check_ref'])"
    done
    for s in 2 3 4; do
      LD_LIBRARY_PATH=$O/lib_$v:${LD_LIBRARY_PATH:-} timeout -k 10 60 opencl-ray-tracer_amd/rt_headless --synthetic 256 64 6.4 \
          --seed 3 --width 4096 --height 4096 --format rgba8 --throughput 600 --inflight $s > $O/cpp_${v}_${s}_$round.txt 2>&1
      rc=$?; [ $rc -ne 0 ] && { cat $O/cpp_${v}_${s}_$round.txt; exit $rc; }
      echo "cpp $v $s $round $(grep -o '[0-9.]* us per frame' $O/cpp_${v}_${s}_$round.txt) $(grep -c 374fec5f43f2decc $O/cpp_${v}_${s}_$round.txt) slots at the fixture hash"
    done
  done
done
echo done
