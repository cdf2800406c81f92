#!/bin/bash
# Round 4: the triangle depth cull in small bands (< 1024 coarse bins), both
# formats, scenes of box overdraw ~5 / ~10 / ~20: library gates vs no
# triangle cull.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=${O:-gpurun_out/r04s}; mkdir -p $O
L=opencl-ray-tracer_amd/librt_hip.so
V="$L $L@coarse_cull_tri=0"
run() { name=$1; shift
  timeout -k 10 200 python scripts/bench_variants.py $V --kernels --rounds 5 "$@" > $O/$name.json 2> $O/$name.err
  rc=$?; echo "$name rc=$rc"; python3 -c "
import json;d=json.load(open('$O/$name.json'))
for k,v in d.items(): print(f\"  {k:32s} frame {v['median_us']:8.2f} bin {v['bin_us']:6.2f} trace {v['trace_us']:8.2f}\")"
  [ $rc -ne 0 ] && { tail -5 $O/$name.err; exit $rc; }; }
for wh in 640x480 1280x720 1920x1080 2560x1440; do
  w=${wh%x*}; h=${wh#*x}
  for sc in 100:100 200:200 400:400; do
    s=${sc%:*}; c=${sc#*:}
    for f in i32x4 rgba8; do run ${wh}_${s}_$f --width $w --height $h --spheres $s --cubes $c --seed 3 --format $f; done
  done
done
echo done
