set -u
cd "${GRAFT_REPO_ROOT}"; mkdir -p gpurun_out; export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m pytest tests -x -q -m gpu -k "golden or device_api or selftest or scene_device or headless or render_multi" --timeout 120 --timeout-method thread > gpurun_out/lazy_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/lazy_tests.log; [ $rc -ne 0 ] && exit $rc
for fmt in i32x4 rgba8; do
timeout -k 10 300 python scripts/inflight_cumask.py --format $fmt --settings 1:ffffffff 2:ffffffff,ffffffff 3:ffffffff,ffffffff,ffffffff 4:ffffffff,ffffffff,ffffffff,ffffffff 2:0fffffff,fffffff0 > gpurun_out/lazy_$fmt.txt 2>&1
rc=$?; echo "$fmt rc=$rc"; cat gpurun_out/lazy_$fmt.txt; [ $rc -ne 0 ] && exit $rc
done
for n in 2 3; do
timeout -k 10 300 python bench.py --steps 40 --warmup 5 --no-cpu-baseline --no-host-path --inflight $n > gpurun_out/lazy_bench$n.json 2> gpurun_out/lazy_bench$n.err
rc=$?; echo "bench $n rc=$rc"; python -c "import json;d=json.load(open('gpurun_out/lazy_bench$n.json'));print(d['ms_per_step'],d['frames_in_flight'],d['one_stream'],d['texture_rgba8']['frames_in_flight'])"; [ $rc -ne 0 ] && exit $rc
done
echo done
