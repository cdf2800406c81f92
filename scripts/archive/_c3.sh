set -e
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
for v in ${VARIANTS:-base c3scan}; do
  cd /tmp
  timeout -k 10 200 rocprofv3 --kernel-trace -d $R/gpurun_out/c3_$v -o run --output-format csv -- python $R/scripts/bench_variants.py $R/opencl-ray-tracer_amd/variants/librt_hip_$v.so --rounds 3 > $R/gpurun_out/c3_$v.log 2>&1
  cd $R
  echo "== $v"; python scripts/gaps.py $(find gpurun_out/c3_$v -name "*kernel_trace.csv" | head -1)
done
