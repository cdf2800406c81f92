#!/bin/bash
# Round 4: the RGBA8 trace's instruction mix, the rehearsal
# tests on the current bench.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r04f; mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_gpu_configs.py -k rehearsal > $O/pytest_rehearsal.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 $O/pytest_rehearsal.log; [ $rc -ne 0 ] && exit $rc
TAG=mix_rgba8 EXTRA="--format rgba8 --no-extras" bash scripts/pmc_mix.sh > $O/mix_rgba8.txt 2>&1 || exit $?

# the 4096-seed randomized parity sweep on this round's library
RT_SWEEP_SEEDS=4096 timeout -k 10 900 python -u -m pytest -q --timeout 120 --timeout-method thread \
    tests/test_gpu_configs.py -k randomized_parity_sweep > $O/parity_sweep_4096.log 2>&1
rc=$?; echo "sweep rc=$rc"; tail -2 $O/parity_sweep_4096.log
echo done
