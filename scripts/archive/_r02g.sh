set -u
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_configs.py -m gpu -k rehearsal > gpurun_out/pt_g.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pt_g.log; [ $rc -ne 0 ] && exit $rc
for n in 2 4; do
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 --master-port 2952$n bench.py --gpus $n --rehearse --steps 10 --warmup 3 --no-extras > gpurun_out/rehearse_g$n.json 2> gpurun_out/rehearse_g$n.err
rc=$?; echo "rehearse $n rc=$rc"; grep "^{" gpurun_out/rehearse_g$n.json | python -c "import json,sys; l=json.loads(sys.stdin.read()); print(l['value'], l['config']['parallelism']); print(json.dumps(l['assembly']))"; [ $rc -ne 0 ] && { tail -20 gpurun_out/rehearse_g$n.err; exit $rc; }
done
exit 0
