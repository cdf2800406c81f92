#!/bin/bash
# Instruction-mix PMC passes for one library variant (LIB=...), kernel-trace only.
# KERNEL=coarse3 aggregates that kernel instead of the trace.
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${TAG:-mix}
export RT_HIP_LIBRARY=${LIB:-$R/opencl-ray-tracer_amd/librt_hip.so}
ARGS="--steps 5 --warmup 2 --no-cpu-baseline --no-host-path ${EXTRA:-}"
i=0
for grp in "SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_CVT SQ_INSTS_VALU_INT64" \
           "SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU" \
           "SQ_WAVES SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_WAIT_ANY SQ_WAIT_INST_ANY" \
           "SQ_INSTS_SMEM SQ_INST_CYCLES_SMEM SQ_INST_LEVEL_SMEM SQ_INSTS_SALU SQ_INSTS_BRANCH SQ_IFETCH" \
           "SQ_INST_CYCLES_VALU SQ_INST_CYCLES_SALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_INSTS_LDS SQ_BUSY_CYCLES"; do
  i=$((i+1))
  (cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --pmc $grp -d "$R/gpurun_out/${TAG}_$i" -o run --output-format csv -- \
      python "$R/bench.py" $ARGS > "$R/gpurun_out/${TAG}_$i.log" 2>&1)
  rc=$?; echo "pass $i rc=$rc"; [ $rc -ne 0 ] && { tail -5 "$R/gpurun_out/${TAG}_$i.log"; exit $rc; }
done
python - "$R/gpurun_out" "$TAG" "${KERNEL:-trace}" <<'PY'
import csv, glob, sys, collections
d, tag, kern = sys.argv[1], sys.argv[2], sys.argv[3]
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(f"{d}/{tag}_*/run_counter_collection.csv"):
    for r in csv.DictReader(open(f)):
        name = r["Kernel_Name"]
        if (kern in name) if kern != "trace" else ("trace3_kernel" in name or "trace_kernel" in name):
            agg["trace"][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, v in sorted(agg["trace"].items()):
    print(f"{k:28s} {sum(v)/len(v):14.0f}")
PY
