#!/bin/bash
# Round 3: RGBA8 renders with the triangle cull in every frame (the new
# default) -- GPU suite, the cull threshold per tile, config 4, the bench line.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out; export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/pytest_tricull.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/pytest_tricull.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python scripts/ab_knob.py --knob coarse_cull_tri --values 4,2,8 --configs c3,c4 --rounds 9 --format rgba8 > gpurun_out/ab_tricull_rgba8_min.jsonl 2>&1 || exit $?
timeout -k 10 300 python scripts/ab_knob.py --knob coarse_cull_overdraw --values 5,0 --configs c4,c5d --rounds 5 --format rgba8 > gpurun_out/ab_tricull_rgba8_gate.jsonl 2>&1 || exit $?
grep -h "^{" gpurun_out/ab_tricull_rgba8_*.jsonl
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-host-path > gpurun_out/bench_tricull.json 2> gpurun_out/bench_tricull.err
rc=$?; echo "bench rc=$rc"; [ $rc -ne 0 ] && { tail -5 gpurun_out/bench_tricull.err; exit $rc; }
python -c "import json;d=json.load(open('gpurun_out/bench_tricull.json'));t=d['texture_rgba8'];print(d['ms_per_step'], t['ms_per_step'], t['one_stream'], t['roofline']['kernel_ms'], t['frames_in_flight'])"
