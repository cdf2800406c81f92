# Frame time vs scene size at 4096^2 (bench.py, N=1, no extras).
set -u
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
for spec in "256 64 6.4" "1024 256 6.4" "4096 1024 6.4" "16384 4096 6.4" "4096 1024 1" "16384 4096 1" "65536 8192 1"; do
  set -- $spec
  timeout -k 10 120 python bench.py --spheres $1 --cubes $2 --k $3 --steps 20 --warmup 3 --no-cpu-baseline --no-host-path --no-extras > gpurun_out/scale_$1_$2_$3.json 2> gpurun_out/scale_$1_$2_$3.err
  rc=$?; [ $rc -ne 0 ] && { echo "$spec rc=$rc"; tail -5 gpurun_out/scale_$1_$2_$3.err; exit $rc; }
  python -c "import json; l=json.load(open('gpurun_out/scale_$1_$2_$3.json')); r=l['roofline']; print('$1 spheres $2 cubes k=$3:', l['ms_per_step'], 'ms', l['value'], 'Mrays/s', 'prep', r['prep_ms'], 'bin', r['bin_ms'], 'trace', r['kernel_ms'], 'frac', r['frac'])"
done
