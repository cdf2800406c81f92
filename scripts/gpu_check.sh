#!/bin/bash
# One GPU session: smoke, GPU parity tests, bench, rocprofv3 kernel stats.
# Stops at the first step that faults / aborts / times out (exit >= 2 from
# pytest counts as a hard failure too); assertion failures in pytest (exit 1)
# are recorded and the measurement steps still run.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r01}
STEPS=${STEPS:-20}
hard_fail() { echo "hard failure ($1) in $2; stopping"; exit "$1"; }

timeout -k 10 240 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; [ $rc -ne 0 ] && { tail -30 gpurun_out/smoke.log; [ $rc -ge 2 ] && hard_fail $rc smoke; }

if [ "${SKIP_TESTS:-0}" != "1" ]; then
  timeout -k 10 600 python -m pytest tests -x -q -m gpu ${PYTEST_ARGS:-} > gpurun_out/pytest_gpu.log 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -15 gpurun_out/pytest_gpu.log
  [ $rc -ge 2 ] && hard_fail $rc pytest
fi

timeout -k 10 300 python bench.py --steps $STEPS --warmup 5 > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err
rc=$?; echo "bench rc=$rc"; cat gpurun_out/bench_$TAG.json; [ $rc -ne 0 ] && { tail -20 gpurun_out/bench_$TAG.err; hard_fail $rc bench; }

if [ "${SKIP_PROF:-0}" != "1" ]; then
  cd /tmp
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/prof_$TAG" -o run --output-format csv -- \
      python "$GRAFT_REPO_ROOT/bench.py" --steps $STEPS --warmup 5 --no-cpu-baseline > "$GRAFT_REPO_ROOT/gpurun_out/prof_$TAG.log" 2>&1
  rc=$?; echo "rocprof rc=$rc"; [ $rc -ne 0 ] && { tail -20 "$GRAFT_REPO_ROOT/gpurun_out/prof_$TAG.log"; hard_fail $rc rocprof; }
  find "$GRAFT_REPO_ROOT/gpurun_out/prof_$TAG" -name "*stats*" | head
fi
echo done
