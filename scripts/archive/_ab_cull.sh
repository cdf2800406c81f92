set -u
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_configs.py -m gpu -k "cull or config5" > gpurun_out/pytest_c.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_c.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python -u scripts/ab_knob.py --knob coarse_cull --values ${VALS:-0,1} --configs ${CFGS:-c3,c5d,c5s,band8,c4} > gpurun_out/ab_cull.jsonl 2>&1
rc=$?; cat gpurun_out/ab_cull.jsonl; exit $rc
