#!/bin/bash
# Round 5: rehearsals N = 2, 4 (scaling_host_frame), the 4096-seed sweep,
# then bench + rocprofv3 on the same build.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r05f; mkdir -p $O
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
for n in 2 4; do
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 --master-port 2950$n \
     bench.py --gpus $n --rehearse --steps 10 --warmup 3 > $O/rehearse_n$n.json 2> $O/rehearse_n$n.err
  rc=$?; echo "rehearse N=$n rc=$rc"; python -c "import json,sys; d=json.load(open('$O/rehearse_n$n.json')); print(d.get('value'), d.get('scaling_host_frame'), d['roofline'].get('frame_frac'), {k: v.get('frame_check') for k, v in d.get('host_frame', {}).items()})"
  [ $rc -ne 0 ] && { tail -20 $O/rehearse_n$n.err; exit $rc; }
done
RT_SWEEP_SEEDS=4096 timeout -k 10 900 python -u -m pytest -q --timeout 120 --timeout-method thread \
    tests/test_gpu_configs.py -k randomized_parity_sweep > $O/parity_sweep_4096.log 2>&1
rc=$?; echo "sweep rc=$rc"; tail -2 $O/parity_sweep_4096.log; [ $rc -ne 0 ] && exit $rc
TAG=r05f SKIP_TESTS=1 bash scripts/gpu_check.sh
