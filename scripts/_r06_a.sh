#!/bin/bash
# Round 6, first GPU session: smoke, the GPU suite (new: config 3 pinned on
# fresh contexts per path, the 4096^2 C++ loop against the fixture, bench.py
# starting its own ranks), the bench line (frame_check_ref, sustained), and
# the C++ loop's slot counts per format at config 3.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r06a; mkdir -p $O
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 240 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; cat $O/smoke.log | tail -5; [ $rc -ne 0 ] && exit $rc
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 240 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 $O/pytest_gpu.log; [ $rc -ge 2 ] && exit $rc
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err
rc=$?; echo "bench rc=$rc"; [ $rc -ne 0 ] && { tail -20 $O/bench.err; exit $rc; }
python - <<'PY'
import json
d = json.load(open("gpurun_out/r06a/bench.json"))
t = d["texture_rgba8"]
print("value", d["value"], "ms", d["ms_per_step"], "ref", d["frame_check_ref"], "frac", d["roofline"]["frame_frac"],
      "sustained", d["frames_in_flight"].get("sustained"))
print("tex", t["value"], t["ms_per_step"], "ref", t["frame_check_ref"], "frac", t["roofline"]["frame_frac"],
      "sustained", (t["frames_in_flight"] or {}).get("sustained"))
PY
export LD_LIBRARY_PATH=$PWD/opencl-ray-tracer_amd:${LD_LIBRARY_PATH:-}
for round in 1 2 3; do
  for fmt in i32x4 rgba8; do
    for s in 2 3; do
      timeout -k 10 60 opencl-ray-tracer_amd/rt_headless --synthetic 256 64 6.4 --seed 3 --width 4096 --height 4096 \
          --format $fmt --throughput 600 --inflight $s > $O/tp_${fmt}_${s}_$round.txt 2>&1
      rc=$?; [ $rc -ne 0 ] && { cat $O/tp_${fmt}_${s}_$round.txt; exit $rc; }
      grep throughput $O/tp_${fmt}_${s}_$round.txt
    done
  done
done
echo done
