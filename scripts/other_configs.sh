#!/bin/bash
# One-GPU bench lines for the BASELINE configs other than the headline
# (config 3), full frames, dense (k = W/640) unless noted; one JSON line each
# into gpurun_out/other_configs.jsonl.  Seeds: config c uses seed c, as the
# tests and bench.py's N>1 config-4 key do.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
OUT=gpurun_out/other_configs.jsonl; : > $OUT
run() {
  timeout -k 10 300 python bench.py --steps ${STEPS:-20} --warmup 5 --no-cpu-baseline --no-host-path "$@" >> $OUT 2> gpurun_out/other_configs.err
  rc=$?; echo "bench $* rc=$rc"; [ $rc -ne 0 ] && { tail -5 gpurun_out/other_configs.err; exit $rc; }
}
run --width 512 --height 512 --spheres 4 --cubes 1 --seed 1           # config 1
run --width 1920 --height 1080 --spheres 16 --cubes 4 --seed 2        # config 2
run --width 1920 --height 1080 --spheres 16 --cubes 4 --seed 2 --format rgba8  # config 2, Texture format
run --width 4096 --height 4096 --spheres 256 --cubes 64 --k 1          # config 3, sparse
run --width 8192 --height 8192 --spheres 192 --cubes 64 --seed 4       # config 4, whole frame
run --width 16384 --height 16384 --spheres 4096 --cubes 0 --seed 5     # config 5, whole frame, dense
run --width 16384 --height 16384 --spheres 4096 --cubes 0 --seed 5 --k 1  # config 5, sparse
run --width 4096 --height 4096 --spheres 256 --cubes 64 --format rgba8 # config 3, Texture format
run --width 16384 --height 16384 --spheres 4096 --cubes 0 --seed 5 --format rgba8  # config 5 dense, Texture
# 8-GPU configs: rank 0's band (weak-scaling layout of bench_variants.py --ranks 8)
L=opencl-ray-tracer_amd/librt_hip.so
band() {
  timeout -k 10 300 python scripts/bench_variants.py $L --rounds 5 "$@" > gpurun_out/band.json 2>>gpurun_out/other_configs.err
  rc=$?; echo "band $* rc=$rc"; [ $rc -ne 0 ] && exit $rc
  python -c "import json,sys; d=json.load(open('gpurun_out/band.json')); print(json.dumps({'band_of_8': sys.argv[1:], 'us_per_frame': list(d.values())[0]['median_us']}))" "$@" >> $OUT
}
band --width 8192 --height 1024 --spheres 24 --cubes 8 --ranks 8 --k 12.8 --seed 4   # config 4: 8192^2 over 8 ranks
band --width 16384 --height 2048 --spheres 512 --cubes 0 --ranks 8 --k 25.6 --seed 5 # config 5: 16384^2 over 8 ranks
echo done
