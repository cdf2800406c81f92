#!/bin/bash
# Round 6: config 5 (16384^2, 4096 spheres) int32x4 in the bench's frame
# loops on three libraries, interleaved, two rounds: the final library
# (base), the same with the verdict copied every 8th launch instead of
# stored by the kernels (vcopy, -DRT_VERDICT_DIRECT=0), and the r06m library
# (commit 370a1a3's rt_device.hip / rt_trace.inc): the other-configs run on
# the final library had config 5's 2-slot loop at 783 us against 675 before.
# (The r06m library, built against the current headers, lacks the new debug
# hook the package binds, so its runs failed; base and vcopy ran: 673 / 617
# us both, i.e. no regression, profiles/r06/c5_check/.)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r06ag; mkdir -p $O
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
V=$PWD/opencl-ray-tracer_amd/variants
for round in 1 2; do
  for v in base vcopy r06m; do
    for k in 25.6 1; do
      RT_HIP_LIBRARY=$V/librt_hip_$v.so timeout -k 10 200 python bench.py --no-host-path --no-cpu-baseline --no-extras \
          --width 16384 --height 16384 --spheres 4096 --cubes 0 --seed 5 --k $k --steps 20 --warmup 5 > $O/c5_${v}_${k}_$round.json 2> $O/c5_${v}_${k}_$round.err
      rc=$?; [ $rc -ne 0 ] && { tail -20 $O/c5_${v}_${k}_$round.err; exit $rc; }
      python -c "
import json; d=json.load(open('$O/c5_${v}_${k}_$round.json')); f=d['frames_in_flight']
print('c5 k=$k $v', $round, 'inflight', f['ms_per_step'], 'sustained', f['sustained']['ms_per_step'], 'one', d['one_stream']['ms_per_step'], 'kernel', d['roofline']['kernel_ms'], f['frame_check'])"
    done
  done
done
echo done
