#!/bin/bash
# Per-wave timeline of the config-3 trace (RT_TIMELINE build), int32x4 and RGBA8.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out; export TMPDIR=/tmp
for f in 0 1; do
  timeout -k 10 200 python scripts/timeline.py opencl-ray-tracer_amd/variants/librt_hip_tl.so 0 $f > gpurun_out/timeline_f$f.txt 2>&1
  rc=$?; echo "== fmt $f rc=$rc"; grep -v amdgpu.ids gpurun_out/timeline_f$f.txt; [ $rc -ne 0 ] && exit $rc
done
echo done
