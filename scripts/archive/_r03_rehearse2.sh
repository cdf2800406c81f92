#!/bin/bash
# Round 3 (final tree): the N>1 bench line rehearsed on one GPU (ranks share
# cuda:0, gloo) at N = 2 and 4, and N = 2 with one assembly forced to fail.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
for n in ${NS:-2 4}; do
  timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 --master-port 2951$n \
     bench.py --gpus $n --rehearse --steps 10 --warmup 3 > gpurun_out/rehearse_r03_n$n.json 2> gpurun_out/rehearse_r03_n$n.err
  rc=$?; echo "rehearse n=$n rc=$rc"; [ $rc -ne 0 ] && { tail -30 gpurun_out/rehearse_r03_n$n.err; exit $rc; }
done
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29519 \
   bench.py --gpus 2 --rehearse --steps 10 --warmup 3 --phase-deadline 30 --fail-assembly xgmi_peer_store:1 > gpurun_out/rehearse_r03_fail.json 2> gpurun_out/rehearse_r03_fail.err
rc=$?; echo "rehearse fail rc=$rc"; [ $rc -ne 0 ] && { tail -30 gpurun_out/rehearse_r03_fail.err; exit $rc; }
echo done
