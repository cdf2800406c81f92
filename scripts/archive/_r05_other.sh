#!/bin/bash
# Round 5: every BASELINE config on the round-5 library (scripts/other_configs.sh),
# plus config 3 int32x4 with 3 frames in flight on CU-masked slot streams.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
bash scripts/other_configs.sh || exit $?
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-host-path --inflight 3 >> gpurun_out/other_configs.jsonl 2>gpurun_out/other_configs.err
rc=$?; echo "c3 3 slots rc=$rc"; exit $rc
