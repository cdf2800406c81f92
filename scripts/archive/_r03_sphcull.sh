#!/bin/bash
# Round 3: the sphere depth-cull gate (sphere candidates per bin) for RGBA8 renders.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python scripts/ab_knob.py --knob coarse_cull --values 10,4,1 --configs c3,c3s,c4 --rounds 9 --format rgba8 > gpurun_out/ab_sphcull_rgba8.jsonl 2>&1 || exit $?
timeout -k 10 300 python scripts/ab_knob.py --knob coarse_cull --values 10,4,1 --configs c3,c5d --rounds 5 > gpurun_out/ab_sphcull_i32.jsonl 2>&1 || exit $?
grep -h "^{" gpurun_out/ab_sphcull_*.jsonl
