#!/bin/bash
# Box-to-box / run-to-run variance of the K=20 window against the long loop:
# the bench twice, then the C++ frame loop at 400 and 4000 frames.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r05var; mkdir -p $O
for i in 1 2; do
  timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --sustained 10 > $O/bench$i.json 2> $O/bench$i.err || exit $?
  python3 -c "import json,sys; d=json.loads(open('$O/bench$i.json').read().splitlines()[-1]); print('bench', d['ms_per_step'], d['frames_in_flight']['sustained']['ms_per_step'], d['texture_rgba8']['ms_per_step'], d['texture_rgba8']['frames_in_flight']['sustained']['ms_per_step'])"
done
export LD_LIBRARY_PATH=opencl-ray-tracer_amd:${LD_LIBRARY_PATH:-}
for f in 20 200 400 4000; do
  timeout -k 10 60 opencl-ray-tracer_amd/rt_headless --synthetic 256 64 6.4 --seed 3 --width 4096 --height 4096 --throughput $f --inflight 2 2>&1 | grep throughput | tee -a $O/headless.txt || exit $?
done
# rocprofv3 of the default bench command (no sustained loop)
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/$O/prof" -o run --output-format csv -- \
    python "$GRAFT_REPO_ROOT/bench.py" --steps 20 --warmup 5 --no-cpu-baseline > "$GRAFT_REPO_ROOT/$O/prof.log" 2>&1 || exit $?
tail -1 "$GRAFT_REPO_ROOT/$O/prof.log"
