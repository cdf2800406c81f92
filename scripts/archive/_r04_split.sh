#!/bin/bash
# Round 4: trace3_split_kernel (2 / 4 waves per wave tile on small frames):
# its parity tests, then A/B against one wave per tile, then the GPU suite
# and the 4096-seed sweep (which now draws the split too).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r04u; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/ \
    -k "split or last_kernel or golden" > $O/pytest_split.log 2>&1
rc=$?; echo "split tests rc=$rc"; tail -3 $O/pytest_split.log; [ $rc -ne 0 ] && exit $rc
L=opencl-ray-tracer_amd/librt_hip.so
V="$L@trace_split=1 $L@trace_split=2 $L@trace_split=4"
run() { name=$1; shift
  timeout -k 10 200 python scripts/bench_variants.py $V --kernels --rounds 5 "$@" > $O/$name.json 2> $O/$name.err
  rc=$?; echo "$name rc=$rc"; python3 -c "
import json;d=json.load(open('$O/$name.json'))
for k,v in d.items(): print(f\"  {k:32s} frame {v['median_us']:8.2f} bin {v['bin_us']:6.2f} trace {v['trace_us']:8.2f}\")"
  [ $rc -ne 0 ] && { tail -5 $O/$name.err; exit $rc; }; }
run scene3 --scene 3
run scene3_rgba8 --scene 3 --format rgba8
for wh in 640x480 1280x720 1920x1080 2560x1440; do
  w=${wh%x*}; h=${wh#*x}
  for sc in 100:100 400:400; do
    s=${sc%:*}; c=${sc#*:}
    run ${wh}_${s} --width $w --height $h --spheres $s --cubes $c --seed 3
  done
done
run 2048_320 --width 2048 --height 2048 --spheres 256 --cubes 64 --seed 3
run 2048_320_rgba8 --width 2048 --height 2048 --spheres 256 --cubes 64 --seed 3 --format rgba8
timeout -k 10 900 python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu tests/ > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $O/pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
RT_SWEEP_SEEDS=4096 timeout -k 10 900 python -u -m pytest -q --timeout 120 --timeout-method thread \
    tests/test_gpu_configs.py -k randomized_parity_sweep > $O/parity_sweep_4096.log 2>&1
rc=$?; echo "sweep rc=$rc"; tail -2 $O/parity_sweep_4096.log
echo done
