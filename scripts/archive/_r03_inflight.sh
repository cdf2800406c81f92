#!/bin/bash
# Round 3: bench.py's N=1 line at 2 / 3 / 4 frames in flight.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
: > gpurun_out/inflight_bench.jsonl
for s in ${SLOTS:-2 3 4}; do
  timeout -k 10 200 python bench.py --steps 40 --warmup 5 --inflight $s --no-cpu-baseline --no-host-path >> gpurun_out/inflight_bench.jsonl 2> gpurun_out/inflight_bench.err || { tail -20 gpurun_out/inflight_bench.err; exit 1; }
done
python3 - <<'PY'
import json
for l in open("gpurun_out/inflight_bench.jsonl"):
    d = json.loads(l)
    f, t = d["frames_in_flight"], d["texture_rgba8"]
    print(f["frames_in_flight"], "i32x4", d["ms_per_step"], d["one_stream"]["ms_per_step"], f["frame_check"],
          "| rgba8", t["ms_per_step"], t["one_stream"]["ms_per_step"], t["frames_in_flight"]["frame_check"])
PY
