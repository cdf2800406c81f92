#!/bin/bash
# GPU session: new config tests, then bench.py N>1 rehearsals (ranks share
# cuda:0, gloo) at N=2 and N=4, then the N=1 bench.  Stops at the first
# hard failure.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
TAG=${TAG:-r02}
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_configs.py ${PYTEST_ARGS:-} > gpurun_out/pytest_cfg_$TAG.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -15 gpurun_out/pytest_cfg_$TAG.log; [ $rc -ne 0 ] && exit $rc
for n in 2 4; do
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 --master-port 2950$n \
     bench.py --gpus $n --rehearse --steps 10 --warmup 3 > gpurun_out/rehearse_${TAG}_$n.json 2> gpurun_out/rehearse_${TAG}_$n.err
  rc=$?; echo "rehearse N=$n rc=$rc"; cat gpurun_out/rehearse_${TAG}_$n.json; [ $rc -ne 0 ] && { tail -30 gpurun_out/rehearse_${TAG}_$n.err; exit $rc; }
done
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err
rc=$?; echo "bench rc=$rc"; cat gpurun_out/bench_$TAG.json; [ $rc -ne 0 ] && { tail -20 gpurun_out/bench_$TAG.err; exit $rc; }
echo done
