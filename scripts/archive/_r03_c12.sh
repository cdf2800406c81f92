set -u
cd "${GRAFT_REPO_ROOT}"; mkdir -p gpurun_out; export TMPDIR=/tmp
for n in 2 3 4; do
 for cfg in "--width 512 --height 512 --spheres 4 --cubes 1 --seed 1" "--width 1920 --height 1080 --spheres 16 --cubes 4 --seed 2"; do
  timeout -k 10 120 python bench.py --steps 40 --warmup 5 --no-cpu-baseline --no-host-path --no-extras --inflight $n $cfg > gpurun_out/c12.json 2>gpurun_out/c12.err
  rc=$?; [ $rc -ne 0 ] && { tail -3 gpurun_out/c12.err; exit $rc; }
  python -c "import json;d=json.load(open('gpurun_out/c12.json'));print($n, d['config']['width'], d['ms_per_step'], d['frames_in_flight'], d['one_stream']['ms_per_step'])"
 done
done
