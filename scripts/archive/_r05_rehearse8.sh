#!/bin/bash
# Round 5 final: N = 8 rehearsal (8 ranks sharing one GPU, gloo) of the
# bench's N>1 phases, to check the world-8 layouts end to end.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r05r8; mkdir -p $O
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29618 \
   bench.py --gpus 8 --rehearse --steps 5 --warmup 2 --no-cpu-baseline > $O/rehearse_n8.json 2> $O/rehearse_n8.err
rc=$?; echo "rehearse N=8 rc=$rc"
python -c "import json; d=json.loads([l for l in open('$O/rehearse_n8.json') if l.startswith('{')][-1]); print(d.get('value'), d.get('ms_per_step'), d.get('scaling_host_frame'), {k: (v.get('ms_per_step'), v.get('frame_check')) for k, v in d.get('assembly', {}).items() if isinstance(v, dict)}, d.get('weak_scaling', {}).get('ms_per_step'))"
exit $rc
