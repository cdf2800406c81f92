#!/bin/bash
# Round 4: first call after rt_reserve; config 4 PMC traffic + instruction
# mix.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r04c; mkdir -p $O
timeout -k 10 120 python scripts/first_call.py --reserve > $O/first_call_reserve.json 2> $O/first_call_reserve.err || exit $?
C4="--width 8192 --height 8192 --spheres 192 --cubes 64 --seed 4"
MODES=0 TAG=c4 BENCH_ARGS="$C4 --steps 10 --warmup 3 --no-cpu-baseline --no-host-path --no-extras" \
  bash scripts/pmc.sh > $O/pmc_c4.txt 2>&1 || exit $?
python scripts/pmc_traffic.py gpurun_out/pmc_c4 $O/pmc_config4.json 8192 8192 192 64 4 i32x4 > $O/pmc_traffic.txt 2>&1
TAG=mix_c4 EXTRA="$C4 --no-extras" bash scripts/pmc_mix.sh > $O/mix_c4.txt 2>&1 || exit $?
TAG=mix_c3 EXTRA="--no-extras" bash scripts/pmc_mix.sh > $O/mix_c3.txt 2>&1 || exit $?
TAG=mix_c5 EXTRA="--width 16384 --height 16384 --spheres 4096 --cubes 0 --seed 5 --no-extras" \
  bash scripts/pmc_mix.sh > $O/mix_c5.txt 2>&1 || exit $?
echo done
