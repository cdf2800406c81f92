#!/bin/bash
# Round 3: coarse workgroups given unused dynamic LDS (rt_debug_set_coarse_lds)
# so fewer coarse waves sit beside the previous frame's trace.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 200 python scripts/inflight.py --slots 1,2 --knob coarse_lds --values 0,14336,34816,60000 --rounds 7 --steps 40 > gpurun_out/clds_i32.txt 2>&1 || { tail gpurun_out/clds_i32.txt; exit 1; }
timeout -k 10 200 python scripts/inflight.py --slots 1,3 --knob coarse_lds --values 0,14336,34816,60000 --rounds 7 --steps 40 --format rgba8 > gpurun_out/clds_rgba8.txt 2>&1 || { tail gpurun_out/clds_rgba8.txt; exit 1; }
grep -hv amdgpu.ids gpurun_out/clds_*.txt
