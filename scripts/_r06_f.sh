#!/bin/bash
# Round 6: the price of one VALU / SALU instruction per wave in the config-3
# trace3_kernel (RGBA8 and int32x4): 50 / 100 extra independent-issue
# instructions per wave (RT_EXTRA_VALU / RT_EXTRA_SALU, diagnostics builds),
# interleaved in one process, frames bit-exact against the base build.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r06f; mkdir -p $O
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
V=opencl-ray-tracer_amd/variants
timeout -k 10 300 python scripts/bench_variants.py $V/librt_hip_base.so $V/librt_hip_v50.so $V/librt_hip_v100.so \
    $V/librt_hip_s50.so $V/librt_hip_s100.so --format rgba8 --kernels --rounds 9 > $O/price_rgba8.json 2> $O/price_rgba8.err
rc=$?; echo "rgba8 rc=$rc"; cat $O/price_rgba8.json; [ $rc -ne 0 ] && { tail -20 $O/price_rgba8.err; exit $rc; }
timeout -k 10 300 python scripts/bench_variants.py $V/librt_hip_base.so@trace_bin=2 $V/librt_hip_v50.so@trace_bin=2 \
    $V/librt_hip_v100.so@trace_bin=2 $V/librt_hip_s50.so@trace_bin=2 $V/librt_hip_s100.so@trace_bin=2 \
    --format i32x4 --kernels --rounds 7 > $O/price_i32x4.json 2> $O/price_i32x4.err
rc=$?; echo "i32x4 rc=$rc"; cat $O/price_i32x4.json; [ $rc -ne 0 ] && { tail -20 $O/price_i32x4.err; exit $rc; }
echo done
