#!/bin/bash
# Round 4, final library: config 3's per-launch HBM traffic (WRITE_SIZE /
# FETCH_SIZE passes, for bench.py's roofline.traffic) and the RGBA8 trace's
# instruction mix.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r04z
TAG=r04z MODES=0 BENCH_ARGS="--steps 10 --warmup 3 --no-cpu-baseline --no-host-path --no-extras" \
    bash scripts/pmc.sh > gpurun_out/r04z/pmc.txt 2>&1 || { tail -5 gpurun_out/r04z/pmc.txt; exit 1; }
cat gpurun_out/r04z/pmc.txt
python scripts/pmc_traffic.py gpurun_out/pmc_r04z gpurun_out/r04z/pmc_config3.json || exit 1
cat gpurun_out/r04z/pmc_config3.json
TAG=mix_rgba8_r04z EXTRA="--format rgba8 --no-extras" bash scripts/pmc_mix.sh > gpurun_out/r04z/mix_rgba8.txt 2>&1 || exit 1
cat gpurun_out/r04z/mix_rgba8.txt
echo done
