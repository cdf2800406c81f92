#!/bin/bash
# Round 4: reference scene 3 at 640x480 (the app's largest scene): the
# coarse kernel with and without its depth-cull stages.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r04p; mkdir -p $O
L=opencl-ray-tracer_amd/librt_hip.so
V="$L $L@coarse_cull_tri=0 $L@coarse_cull=0,coarse_cull_tri=0"
for f in i32x4 rgba8; do
  timeout -k 10 200 python scripts/bench_variants.py $V --scene 3 --format $f --kernels --rounds 7 \
      > $O/s3_$f.json 2> $O/s3_$f.err
  rc=$?; echo "s3 $f rc=$rc"; cat $O/s3_$f.json; [ $rc -ne 0 ] && { tail -5 $O/s3_$f.err; exit $rc; }
done
echo done
