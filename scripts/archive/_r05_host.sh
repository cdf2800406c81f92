#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r05host; mkdir -p $O
timeout -k 10 200 python scripts/host_rate.py > $O/host_rate.txt 2>&1; rc=$?; grep -v amdgpu $O/host_rate.txt; [ $rc -ne 0 ] && exit $rc
export LD_LIBRARY_PATH=opencl-ray-tracer_amd:${LD_LIBRARY_PATH:-}
for a in "--inflight 2" "--inflight 1" "--inflight 3 --format rgba8" "--inflight 2 --format rgba8"; do
  timeout -k 10 60 opencl-ray-tracer_amd/rt_headless --synthetic 256 64 6.4 --seed 3 --width 4096 --height 4096 --throughput 400 $a 2>&1 | grep throughput | tee -a $O/headless.txt
done
