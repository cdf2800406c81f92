#!/bin/bash
# Round 3: frame_small_kernel with several wave tiles per wave (rt_debug_set_small_tiles).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 200 python scripts/ab_knob.py --knob small_tiles --values 1,2,3,4,8 --configs c1,c2,s2 --rounds 9 --steps 40 > gpurun_out/ab_stiles_i32.jsonl 2>&1 || { tail gpurun_out/ab_stiles_i32.jsonl; exit 1; }
timeout -k 10 200 python scripts/ab_knob.py --knob small_tiles --values 1,2,3,4,8 --configs c2 --rounds 9 --steps 40 --format rgba8 > gpurun_out/ab_stiles_rgba8.jsonl 2>&1 || { tail gpurun_out/ab_stiles_rgba8.jsonl; exit 1; }
timeout -k 10 200 python scripts/ab_knob.py --knob small_tiles --values 1,2,4,8,16 --configs uhd64,c3s64,c3s16 --rounds 5 --steps 20 --fixed small_fused=2 > gpurun_out/ab_stiles_big.jsonl 2>&1 || { tail gpurun_out/ab_stiles_big.jsonl; exit 1; }
timeout -k 10 200 python scripts/ab_knob.py --knob small_fused --values 0,1 --configs uhd64,c3s64,c3s16 --rounds 5 --steps 20 > gpurun_out/ab_stiles_ref.jsonl 2>&1 || { tail gpurun_out/ab_stiles_ref.jsonl; exit 1; }
grep -h "^{" gpurun_out/ab_stiles_*.jsonl
