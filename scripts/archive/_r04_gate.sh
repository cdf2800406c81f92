#!/bin/bash
# Round 4: where the RGBA8 renders' triangle depth cull (coarse kernel) pays:
# frame sizes x scenes, default gate vs none.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=${O:-gpurun_out/r04q}; mkdir -p $O
L=opencl-ray-tracer_amd/librt_hip.so
V="$L $L@coarse_cull_tri=0"
run() { name=$1; shift
  timeout -k 10 200 python scripts/bench_variants.py $V --format rgba8 --kernels --rounds 5 "$@" > $O/$name.json 2> $O/$name.err
  rc=$?; echo "$name rc=$rc"; python3 -c "
import json;d=json.load(open('$O/$name.json'))
for k,v in d.items(): print(f\"  {k:32s} frame {v['median_us']:8.2f} bin {v['bin_us']:6.2f} trace {v['trace_us']:8.2f}\")"
  [ $rc -ne 0 ] && { tail -5 $O/$name.err; exit $rc; }; }
run s3 --scene 3
run s3_i32x4 --scene 3 --format i32x4
for wh in 640x480 1280x720 1920x1080 2560x1440 3840x2160 4096x4096; do
  w=${wh%x*}; h=${wh#*x}
  run ${wh}_200 --width $w --height $h --spheres 100 --cubes 100 --seed 3
  run ${wh}_320 --width $w --height $h --spheres 256 --cubes 64 --seed 3
done
echo done
