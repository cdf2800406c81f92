#!/bin/bash
# Round-3 checkpoint on one GPU: smoke, the GPU suite, the N=1 bench line,
# rocprofv3 kernel stats of the same bench.  Stops at the first step that
# faults, aborts or times out.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
T=${TAG:-r03}
timeout -k 10 240 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$T.log 2>&1
rc=$?; echo "smoke rc=$rc"; [ $rc -ne 0 ] && { tail -20 gpurun_out/smoke_$T.log; exit $rc; }
if [ "${SKIP_TESTS:-0}" != 1 ]; then
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/pytest_$T.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -8 gpurun_out/pytest_$T.log; [ $rc -ge 2 ] && exit $rc
fi
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_$T.json 2> gpurun_out/bench_$T.err
rc=$?; echo "bench rc=$rc"; cat gpurun_out/bench_$T.json | cut -c1-600; [ $rc -ne 0 ] && { tail -20 gpurun_out/bench_$T.err; exit $rc; }
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/prof_$T" -o run --output-format csv -- \
    python "$GRAFT_REPO_ROOT/bench.py" --steps 20 --warmup 5 --no-cpu-baseline --no-host-path > "$GRAFT_REPO_ROOT/gpurun_out/prof_$T.log" 2>&1
rc=$?; echo "rocprof rc=$rc"; [ $rc -ne 0 ] && { tail -20 "$GRAFT_REPO_ROOT/gpurun_out/prof_$T.log"; exit $rc; }
echo done
