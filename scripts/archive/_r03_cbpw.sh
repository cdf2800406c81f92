#!/bin/bash
# Round 3: coarse kernel with several bins per wave (fewer coarse waves beside
# the previous frame's trace), frames in flight and one stream; wave launch rate.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 200 python scripts/inflight.py --slots 1,2 --cbpw 1,2,4,8 --rounds 7 --steps 40 > gpurun_out/cbpw_i32.txt 2>&1 || { tail gpurun_out/cbpw_i32.txt; exit 1; }
cat gpurun_out/cbpw_i32.txt
timeout -k 10 200 python scripts/inflight.py --slots 1,3 --cbpw 1,2,4,8 --rounds 7 --steps 40 --format rgba8 > gpurun_out/cbpw_rgba8.txt 2>&1 || { tail gpurun_out/cbpw_rgba8.txt; exit 1; }
cat gpurun_out/cbpw_rgba8.txt
timeout -k 10 200 python scripts/ab_knob.py --knob coarse_bins_per_wave --values 1,2,4,8 --configs c3,c4,c5d --rounds 5 > gpurun_out/ab_cbpw.jsonl 2>&1 || { tail gpurun_out/ab_cbpw.jsonl; exit 1; }
grep -h "^{" gpurun_out/ab_cbpw.jsonl
timeout -k 10 60 ./scripts/wave_rate > gpurun_out/wave_rate.txt 2>&1 && cat gpurun_out/wave_rate.txt
