#!/bin/bash
# Round 3: the N>1 bench paths on one GPU (rehearsal), the forced-failure
# line, then the N=1 bench line.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 500 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_gpu_configs.py -k "rehearsal" > gpurun_out/pytest_rehearsal.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -6 gpurun_out/pytest_rehearsal.log; [ $rc -ge 2 ] && exit $rc
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29502 \
   bench.py --gpus 2 --rehearse --steps 10 --warmup 3 > gpurun_out/rehearse_r03_2.json 2> gpurun_out/rehearse_r03_2.err
rc=$?; echo "rehearse rc=$rc"; [ $rc -ne 0 ] && { tail -30 gpurun_out/rehearse_r03_2.err; exit $rc; }
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_r03a.json 2> gpurun_out/bench_r03a.err
rc=$?; echo "bench rc=$rc"; cat gpurun_out/bench_r03a.json; [ $rc -ne 0 ] && { tail -20 gpurun_out/bench_r03a.err; exit $rc; }
echo done
