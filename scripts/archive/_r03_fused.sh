#!/bin/bash
# Round 3: prep + coarse fused into one kernel (bin_fused_kernel) vs the
# two-kernel path, interleaved A/B with frame checks, then the GPU suite.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python scripts/ab_knob.py --knob fused_bin --values 0,1 --configs ${C_I32:-c3,c3s,c4,c4band,p512} > gpurun_out/ab_fused_i32.jsonl 2>&1
rc=$?; echo "ab i32 rc=$rc"; [ $rc -ge 124 ] && exit $rc
timeout -k 10 300 python scripts/ab_knob.py --knob fused_bin --values 0,1 --format rgba8 --configs ${C_RGBA:-c3,c4} > gpurun_out/ab_fused_rgba8.jsonl 2>&1
rc=$?; echo "ab rgba8 rc=$rc"; [ $rc -ge 124 ] && exit $rc
if [ "${SKIP_TESTS:-0}" != 1 ]; then
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 240 --timeout-method thread > gpurun_out/pytest_fused.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/pytest_fused.log
fi
timeout -k 10 200 python scripts/ref_kernel_default_build.py > gpurun_out/reference_kernel_default_build.jsonl 2> gpurun_out/refdef.err
echo "refdef rc=$?"
exit 0
