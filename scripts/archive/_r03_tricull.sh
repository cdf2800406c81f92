#!/bin/bash
# Round 3: the triangle depth cull on the BASELINE configs regardless of the
# frame's box overdraw (gate 0) vs the default gate (5), and the per-bin
# candidate threshold at gate 0.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python scripts/ab_knob.py --knob coarse_cull_overdraw --values 5,0 --configs c3,c3s,c4 --rounds 9 > gpurun_out/ab_tricull_gate.jsonl 2>&1 || exit $?
timeout -k 10 300 python scripts/ab_knob.py --knob coarse_cull_overdraw --values 5,0 --configs c3 --rounds 9 --format rgba8 > gpurun_out/ab_tricull_gate_rgba8.jsonl 2>&1 || exit $?
timeout -k 10 300 python scripts/ab_knob.py --knob coarse_cull_tri --values 4,2,1 --fixed coarse_cull_overdraw=0 --configs c3,c4 --rounds 9 > gpurun_out/ab_tricull_min.jsonl 2>&1 || exit $?
grep -h "^{" gpurun_out/ab_tricull_*.jsonl
