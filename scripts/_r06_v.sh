#!/bin/bash
# Round 6, final library (the overdraw verdict written by the kernels into
# the host word; trace_bin_kernel.s arguments reordered for preloading): smoke, the GPU suite, the 4096-seed sweep, an N = 2
# rehearsal through bench.py's own launcher, the default bench line, its
# rocprofv3 kernel trace + stats (--sustained 0), the trace kernel's HBM
# traffic, and the C++ frame loop at config 3.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r06v; mkdir -p $O
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 240 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -3 $O/smoke.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 240 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $O/pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
RT_SWEEP_SEEDS=4096 timeout -k 10 600 python -u -m pytest -q --timeout 120 --timeout-method thread \
    tests/test_gpu_configs.py -k randomized_parity_sweep > $O/parity_sweep_4096.log 2>&1
rc=$?; echo "sweep rc=$rc"; tail -1 $O/parity_sweep_4096.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python bench.py --gpus 2 --rehearse --steps 10 --warmup 3 > $O/rehearse_n2.json 2> $O/rehearse_n2.err
rc=$?; echo "rehearse rc=$rc"; [ $rc -ne 0 ] && { tail -20 $O/rehearse_n2.err; exit $rc; }
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err
rc=$?; echo "bench rc=$rc"; [ $rc -ne 0 ] && { tail -20 $O/bench.err; exit $rc; }
python - <<'PY'
import json
d = json.load(open("gpurun_out/r06v/bench.json"))
t = d["texture_rgba8"]
print("value", d["value"], d["ms_per_step"], d["frame_check_ref"], d["roofline"]["frac"], d["roofline"]["frame_frac"],
      d["roofline"]["kernel_ms"], d["frames_in_flight"]["sustained"])
print("tex", t["value"], t["ms_per_step"], t["frame_check_ref"], t["roofline"]["frame_frac"], t["roofline"]["kernel_ms"],
      t["frames_in_flight"]["sustained"])
r = json.loads(open("gpurun_out/r06v/rehearse_n2.json").read())
print("rehearse", r["value"], r["scaling_assembled"], r["scaling_weak"], {k: (v.get("frame_check"), v.get("frame_check_ref")) for k, v in r["assembly"].items()})
PY
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/$O/prof" -o run --output-format csv -- \
    python "$GRAFT_REPO_ROOT/bench.py" --steps 20 --warmup 5 --sustained 0 > "$GRAFT_REPO_ROOT/$O/prof_bench.json" 2> "$GRAFT_REPO_ROOT/$O/prof_bench.err"
rc=$?; echo "rocprof rc=$rc"; [ $rc -ne 0 ] && { tail -20 "$GRAFT_REPO_ROOT/$O/prof_bench.err"; exit $rc; }
i=0
for grp in WRITE_SIZE FETCH_SIZE; do
  i=$((i+1))
  timeout -k 10 200 rocprofv3 --kernel-trace --pmc $grp -d "$GRAFT_REPO_ROOT/$O/pmc_$i" -o run --output-format csv -- \
      python "$GRAFT_REPO_ROOT/bench.py" --steps 10 --warmup 3 --no-cpu-baseline --no-host-path --no-extras \
      --sustained 0 > "$GRAFT_REPO_ROOT/$O/pmc_$i.log" 2>&1
  rc=$?; echo "pmc pass $i ($grp) rc=$rc"; [ $rc -ne 0 ] && { tail -8 "$GRAFT_REPO_ROOT/$O/pmc_$i.log"; exit $rc; }
done
cd "$GRAFT_REPO_ROOT"
python scripts/rocprof_launches.py $O/prof/run_kernel_trace.csv trace_bin_kernel
export LD_LIBRARY_PATH=$PWD/opencl-ray-tracer_amd:${LD_LIBRARY_PATH:-}
for fmt in i32x4 rgba8; do
  timeout -k 10 60 opencl-ray-tracer_amd/rt_headless --synthetic 256 64 6.4 --seed 3 --width 4096 --height 4096 \
      --format $fmt --throughput 600 --inflight 2 > $O/cpp_$fmt.txt 2>&1
  rc=$?; cat $O/cpp_$fmt.txt | grep -E "throughput|slot"; [ $rc -ne 0 ] && exit $rc
done
echo done
