#!/bin/bash
# Round 4: GPU suite, the N>1 bench paths on one GPU (rehearsal: N = 2, 4,
# both host-frame formats with their one-GPU ratio), then the N=1 line.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; O=gpurun_out/r04d; mkdir -p $O
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 900 python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu tests/ > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -6 $O/pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
for n in 2 4; do
  timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 \
     --master-port 2951$n bench.py --gpus $n --rehearse --steps 10 --warmup 3 > $O/rehearse_n$n.json 2> $O/rehearse_n$n.err
  rc=$?; echo "rehearse n=$n rc=$rc"; [ $rc -ne 0 ] && { tail -30 $O/rehearse_n$n.err; exit $rc; }
done
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err
rc=$?; echo "bench rc=$rc"; [ $rc -ne 0 ] && { tail -20 $O/bench.err; exit $rc; }
echo done
