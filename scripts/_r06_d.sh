#!/bin/bash
# Round 6: N = 2 / 4 / 8 rehearsals through bench.py's own launcher (no
# torchrun; ranks share cuda:0, gloo), the 4096-seed parity sweep on this
# library, the default bench line, its rocprofv3 kernel trace + stats, and
# the trace kernel's HBM traffic (WRITE_SIZE / FETCH_SIZE, separate passes).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r06d; mkdir -p $O
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
for n in 2 4 8; do
  timeout -k 10 500 python bench.py --gpus $n --rehearse --steps 10 --warmup 3 > $O/rehearse_n$n.json 2> $O/rehearse_n$n.err
  rc=$?; echo "rehearse N=$n rc=$rc"; [ $rc -ne 0 ] && { tail -20 $O/rehearse_n$n.err; exit $rc; }
  python -c "
import json; d=json.load(open('$O/rehearse_n$n.json'))
print(d['value'], d['scaling_assembled'], d['scaling_weak'], d['scaling_host_frame'], {k: (v.get('frame_check'), v.get('frame_check_ref')) for k, v in d['assembly'].items()})"
done
RT_SWEEP_SEEDS=4096 timeout -k 10 600 python -u -m pytest -q --timeout 120 --timeout-method thread \
    tests/test_gpu_configs.py -k randomized_parity_sweep > $O/parity_sweep_4096.log 2>&1
rc=$?; echo "sweep rc=$rc"; tail -2 $O/parity_sweep_4096.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err
rc=$?; echo "bench rc=$rc"; [ $rc -ne 0 ] && { tail -20 $O/bench.err; exit $rc; }
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/$O/prof" -o run --output-format csv -- \
    python "$GRAFT_REPO_ROOT/bench.py" --steps 20 --warmup 5 > "$GRAFT_REPO_ROOT/$O/prof_bench.json" 2> "$GRAFT_REPO_ROOT/$O/prof_bench.err"
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
find $O/prof -name "*stats*" | head
python - <<'PY'
import json
d = json.load(open("gpurun_out/r06d/bench.json"))
t = d["texture_rgba8"]
print("value", d["value"], d["ms_per_step"], d["frame_check_ref"], d["roofline"]["frac"], d["roofline"]["frame_frac"],
      d["frames_in_flight"]["sustained"])
print("tex", t["value"], t["ms_per_step"], t["frame_check_ref"], t["roofline"]["frame_frac"], t["frames_in_flight"]["sustained"])
PY
echo done
