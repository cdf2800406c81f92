set -u
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_configs.py -m gpu > gpurun_out/pt_d.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pt_d.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29512 bench.py --gpus 2 --rehearse --steps 10 --warmup 3 > gpurun_out/rehearse_d2.json 2> gpurun_out/rehearse_d2.err
rc=$?; echo "rehearse rc=$rc"; cat gpurun_out/rehearse_d2.json; [ $rc -ne 0 ] && { tail -20 gpurun_out/rehearse_d2.err; exit $rc; }
timeout -k 10 300 python bench.py > gpurun_out/bench_d.json 2> gpurun_out/bench_d.err
rc=$?; echo "bench rc=$rc"; cat gpurun_out/bench_d.json; [ $rc -ne 0 ] && { tail -20 gpurun_out/bench_d.err; exit $rc; }
exit 0
