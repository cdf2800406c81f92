#!/bin/bash
# One-GPU bench lines for the BASELINE configs other than the headline
# (config 3), full frames, dense (k = W/640) unless noted; one JSON line each
# into gpurun_out/other_configs.jsonl.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
OUT=gpurun_out/other_configs.jsonl; : > $OUT
run() {
  timeout -k 10 300 python bench.py --steps ${STEPS:-20} --warmup 5 --no-cpu-baseline --no-host-path "$@" >> $OUT 2> gpurun_out/other_configs.err
  rc=$?; echo "bench $* rc=$rc"; [ $rc -ne 0 ] && { tail -5 gpurun_out/other_configs.err; exit $rc; }
}
run --width 1920 --height 1080 --spheres 16 --cubes 4                 # config 2
run --width 4096 --height 4096 --spheres 256 --cubes 64 --k 1          # config 3, sparse
run --width 8192 --height 8192 --spheres 192 --cubes 64                # config 4, whole frame
run --width 16384 --height 16384 --spheres 4096 --cubes 0              # config 5, whole frame, dense
run --width 16384 --height 16384 --spheres 4096 --cubes 0 --k 1        # config 5, sparse
run --width 4096 --height 4096 --spheres 256 --cubes 64 --format rgba8 # config 3, Texture format
echo done
