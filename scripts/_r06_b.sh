#!/bin/bash
# Round 6: the 8-rows-per-lane trace (16x32 tiles in the 16x16 build,
# coordinates re-derived per use, rows in groups of 2: 63 VGPRs, no VGPR
# spill for the RGBA8 trace) against the shipped build, interleaved in one
# process (scripts/bench_variants.py), then the frame loop and the PMC mix.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r06b; mkdir -p $O
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
V=opencl-ray-tracer_amd/variants
timeout -k 10 300 python scripts/bench_variants.py $V/librt_hip_base.so $V/librt_hip_r8g2.so $V/librt_hip_r4fresh.so \
    --format rgba8 --kernels --rounds 9 > $O/ab_rgba8.json 2> $O/ab_rgba8.err
rc=$?; echo "ab rgba8 rc=$rc"; cat $O/ab_rgba8.json; [ $rc -ne 0 ] && { tail -20 $O/ab_rgba8.err; exit $rc; }
timeout -k 10 300 python scripts/bench_variants.py $V/librt_hip_base.so@trace_bin=2 $V/librt_hip_r8g2.so@trace_bin=2 \
    $V/librt_hip_r4fresh.so@trace_bin=2 $V/librt_hip_base.so \
    --format i32x4 --kernels --rounds 7 > $O/ab_i32x4.json 2> $O/ab_i32x4.err
rc=$?; echo "ab i32x4 rc=$rc"; cat $O/ab_i32x4.json; [ $rc -ne 0 ] && { tail -20 $O/ab_i32x4.err; exit $rc; }
for v in base r8g2; do
  for s in 2 3; do
    RT_HIP_LIBRARY=$PWD/$V/librt_hip_$v.so timeout -k 10 200 python bench.py --format rgba8 --no-extras --no-host-path \
        --no-cpu-baseline --inflight $s --steps 20 --warmup 5 --sustained 600 > $O/frame_${v}_$s.json 2> $O/frame_${v}_$s.err
    rc=$?; [ $rc -ne 0 ] && { tail -20 $O/frame_${v}_$s.err; exit $rc; }
    python -c "import json; d=json.load(open('$O/frame_${v}_$s.json')); f=d['frames_in_flight']; print('$v', $s, d['ms_per_step'], d['roofline']['kernel_ms'], f and f.get('sustained'), d['frame_check_ref'])"
  done
done
for v in base r8g2; do
  i=0
  for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_WAIT_ANY SQ_WAIT_INST_ANY" \
             "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_IFETCH SQ_INSTS_VALU_MUL_F64"; do
    i=$((i+1))
    (cd /tmp && RT_HIP_LIBRARY=$GRAFT_REPO_ROOT/$V/librt_hip_$v.so timeout -k 10 200 rocprofv3 --kernel-trace --pmc $grp \
        -d "$GRAFT_REPO_ROOT/$O/pmc_${v}_$i" -o run --output-format csv -- \
        python "$GRAFT_REPO_ROOT/bench.py" --format rgba8 --no-extras --no-host-path --no-cpu-baseline --inflight 1 \
        --sustained 0 --steps 10 --warmup 3 > "$GRAFT_REPO_ROOT/$O/pmc_${v}_$i.log" 2>&1)
    rc=$?; echo "pmc $v pass $i rc=$rc"; [ $rc -ne 0 ] && { tail -5 "$O/pmc_${v}_$i.log"; exit $rc; }
  done
done
python - <<'PY'
import csv, glob, collections
for v in ("base", "r8g2"):
    agg = collections.defaultdict(list)
    for f in glob.glob(f"gpurun_out/r06b/pmc_{v}_*/run_counter_collection.csv"):
        for r in csv.DictReader(open(f)):
            if "trace3_kernel" in r["Kernel_Name"]:
                agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
    print(v, {k: round(sum(x) / len(x)) for k, x in sorted(agg.items())})
PY
echo done
