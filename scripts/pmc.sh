#!/bin/bash
# PMC passes (one counter group per rocprofv3 run, kernel-trace only, as
# MI355X_MICROARCH.md's rocprofv3 section prescribes) + ablation timings.
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${TAG:-r01}
ARGS=${BENCH_ARGS:-"--steps 10 --warmup 3 --no-cpu-baseline"}
for mode in ${MODES:-0}; do  # 1 2: ablations, RT_DIAG=1 library only
  timeout -k 10 200 python bench.py $ARGS --trace-mode $mode > gpurun_out/ablate_${TAG}_m$mode.json 2>gpurun_out/ablate_${TAG}_m$mode.err
  rc=$?; echo "ablation mode $mode rc=$rc"; cat gpurun_out/ablate_${TAG}_m$mode.json
  [ $rc -ne 0 ] && { tail -5 gpurun_out/ablate_${TAG}_m$mode.err; exit $rc; }
done
i=0
for grp in "WRITE_SIZE" "FETCH_SIZE" \
           "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS GRBM_GUI_ACTIVE" \
           "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU" \
           "SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_INST_CYCLES_VMEM_WR"; do
  i=$((i+1))
  (cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --pmc $grp -d "$R/gpurun_out/pmc_${TAG}_$i" -o run --output-format csv -- \
      python "$R/bench.py" $ARGS > "$R/gpurun_out/pmc_${TAG}_$i.log" 2>&1)
  rc=$?; echo "pmc pass $i ($grp) rc=$rc"
  [ $rc -ne 0 ] && { tail -8 "$R/gpurun_out/pmc_${TAG}_$i.log"; [ $rc -ge 124 ] && exit $rc; }
done
echo done
