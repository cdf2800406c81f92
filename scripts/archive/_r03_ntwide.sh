#!/bin/bash
# Round 3: with nontemporal stores in the wide build, the 16x16 build (1) vs
# the wide build (2) on frames below the wide build's 512 MiB threshold.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 200 python scripts/ab_knob.py --knob tile_variant --values 1,2 --configs c3,c3s,band8,c4half --rounds 7 > gpurun_out/ntwide_i32.jsonl 2>&1 || { tail gpurun_out/ntwide_i32.jsonl; exit 1; }
timeout -k 10 200 python scripts/ab_knob.py --knob tile_variant --values 1,2 --configs c3,c4 --rounds 7 --format rgba8 > gpurun_out/ntwide_rgba8.jsonl 2>&1 || { tail gpurun_out/ntwide_rgba8.jsonl; exit 1; }
grep -h "^{" gpurun_out/ntwide_*.jsonl
