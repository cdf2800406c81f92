#!/bin/bash
# Round 4: coarse3_kernel with 2 / 4 waves per bin on bands of few bins: its
# parity tests first, then A/B against one wave per bin, then the GPU suite
# and the 4096-seed sweep (which draws the coarse waves too).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r04v; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/ \
    -k "coarse_waves or split or golden or depth_cull" > $O/pytest_cw.log 2>&1
rc=$?; echo "cw tests rc=$rc"; tail -3 $O/pytest_cw.log; [ $rc -ne 0 ] && exit $rc
L=opencl-ray-tracer_amd/librt_hip.so
V="$L@coarse_waves=1 $L@coarse_waves=2 $L@coarse_waves=4"
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
run c3 --rounds 5
run c3_rgba8 --format rgba8
run c5 --width 16384 --height 16384 --spheres 4096 --cubes 0 --seed 5 --rounds 3 --steps 5
timeout -k 10 900 python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu tests/ > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $O/pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
RT_SWEEP_SEEDS=4096 timeout -k 10 900 python -u -m pytest -q --timeout 120 --timeout-method thread \
    tests/test_gpu_configs.py -k randomized_parity_sweep > $O/parity_sweep_4096.log 2>&1
rc=$?; echo "sweep rc=$rc"; tail -2 $O/parity_sweep_4096.log
echo done
