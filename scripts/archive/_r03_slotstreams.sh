set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
for ss in ${SS:-hip cumask hip cumask}; do
  timeout -k 10 200 python bench.py --steps 40 --warmup 5 --no-cpu-baseline --no-host-path --slot-streams $ss > gpurun_out/ss_$ss.json 2> gpurun_out/ss_$ss.err
  rc=$?; [ $rc -ne 0 ] && { tail -5 gpurun_out/ss_$ss.err; exit $rc; }
  python -c "import json;d=json.load(open('gpurun_out/ss_$ss.json'));t=d['texture_rgba8'];print('$ss', 'i32', d['frames_in_flight']['ms_per_step'], d['one_stream']['ms_per_step'], 'rgba8', t['frames_in_flight']['ms_per_step'], t['one_stream']['ms_per_step'], t['roofline']['kernel_ms'])"
done
