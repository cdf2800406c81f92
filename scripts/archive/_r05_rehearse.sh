#!/bin/bash
# Round 5 final: N = 2 / 4 rehearsals (ranks sharing one GPU) on the bench
# whose timed windows each follow a per-rank clock ramp.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r05j; mkdir -p $O
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
for n in 2 4; do
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 --master-port 2960$n \
     bench.py --gpus $n --rehearse --steps 10 --warmup 3 > $O/rehearse_n$n.json 2> $O/rehearse_n$n.err
  rc=$?; echo "rehearse N=$n rc=$rc"; python -c "import json,sys; d=json.load(open('$O/rehearse_n$n.json')); print(d.get('value'), d.get('ms_per_step'), d.get('scaling_host_frame'), d['roofline'].get('frame_frac'), {k: (v.get('ms_per_step'), v.get('frame_check')) for k, v in d.get('assembly', {}).items() if isinstance(v, dict)})"
  [ $rc -ne 0 ] && { tail -20 $O/rehearse_n$n.err; exit $rc; }
done
