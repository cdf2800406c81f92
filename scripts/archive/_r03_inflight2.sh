#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
timeout -k 10 200 python scripts/inflight_cumask.py --rounds 9 --settings "1:ffffffff" "2:ffffffff,ffffffff" "3:ffffffff,ffffffff,ffffffff" "2:0fffffff,fffffff0" > gpurun_out/inflight_cumask2.txt 2>&1 || exit 1
SLOTS="2 3 2 3" bash scripts/_r03_inflight.sh
