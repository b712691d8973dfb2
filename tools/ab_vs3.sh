# A/B of libgsr variants (tools/ab/libgsr_<v>.so) in the default 3-stream step only, alternated
# over 3 reps; prints value and the concurrent + solo binning phase times.  usage: bash tools/ab_vs3.sh a b ...
set -o pipefail
mkdir -p gpurun_out/ab3
for rep in ${REPS:-1 2 3}; do
  for v in "$@"; do
    GSR_LIB=$(pwd)/tools/ab/libgsr_$v.so timeout -k 10 200 python -u bench.py --steps ${STEPS:-60} ${BENCH_ARGS:-} \
      --call-site-steps 0 --loss-steps 0 --densify-steps 0 --io-timesteps 0 --no-cpu-baseline \
      > gpurun_out/ab3/$v.$rep.json 2> gpurun_out/ab3/$v.$rep.err || { echo "$v failed"; tail -5 gpurun_out/ab3/$v.$rep.err; exit 1; }
    python -c "
import json; d=json.loads([l for l in open('gpurun_out/ab3/$v.$rep.json') if l.startswith('{')][0])
p=d['phase_ms_per_launch']; s=d['phase_ms_per_launch_solo']
print('$v rep=$rep', d['value'], d['ms_per_step'], {k: (round(s[k]*1e3), round(p[k]*1e3)) for k in ('bin_count','bin_emit','render_fwd','render_bwd')})"
  done
done
