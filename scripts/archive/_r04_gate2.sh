#!/bin/bash
# Round 4: the RGBA8 triangle-cull frame-size gate -- the sweep again on the
# gated library, then the GPU suite.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r04r bash scripts/_r04_gate.sh || exit $?
timeout -k 10 900 python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu tests/ > gpurun_out/r04r/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/r04r/pytest_gpu.log; exit $rc
