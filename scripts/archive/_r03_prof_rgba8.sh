#!/bin/bash
# rocprofv3 kernel stats of the config-3 Texture (RGBA8) frame rendered on one
# stream (no frames in flight, so no other frame's prep / coarse kernels run
# beside the trace and stretch its duration).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out; export TMPDIR=/tmp
R="$GRAFT_REPO_ROOT"
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_rgba8" -o run --output-format csv -- \
    python "$R/bench.py" --steps 50 --warmup 5 --format rgba8 --inflight 1 --no-extras --no-cpu-baseline --no-host-path > "$R/gpurun_out/prof_rgba8.log" 2>&1
rc=$?; echo "rocprof rgba8 rc=$rc"; [ $rc -ne 0 ] && { tail -20 "$R/gpurun_out/prof_rgba8.log"; exit $rc; }
head -c 700 "$R/gpurun_out/prof_rgba8.log"; echo
