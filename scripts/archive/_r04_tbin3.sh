#!/bin/bash
# Round 4 experiment: the no-coarse trace on int32x4 frames of high box
# overdraw (config 3's scene at 2x / 4x object size), one stream.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r04tb3; mkdir -p $O
L=opencl-ray-tracer_amd/librt_hip.so
V="$L $L@trace_bin=1"
run() { name=$1; shift
  timeout -k 10 300 python scripts/bench_variants.py $V --kernels --rounds 5 "$@" > $O/$name.json 2> $O/$name.err
  rc=$?; echo "$name rc=$rc"; python3 -c "
import json;d=json.load(open('$O/$name.json'))
for k,v in d.items(): print(f\"  {k:32s} frame {v['median_us']:8.2f} prep {v['prep_us']:6.2f} bin {v['bin_us']:6.2f} trace {v['trace_us']:8.2f}\")"
  [ $rc -ne 0 ] && { tail -5 $O/$name.err; exit $rc; }; }
run c3_k12 --k 12.8
run c3_k25 --k 25.6
run c3_k51 --k 51.2
run c3_spheres1000 --spheres 1000 --cubes 2 --k 12.8
run 2560x1440 --width 2560 --height 1440 --spheres 256 --cubes 64 --seed 3
run 3840x2160 --width 3840 --height 2160 --spheres 256 --cubes 64 --seed 3
echo done
