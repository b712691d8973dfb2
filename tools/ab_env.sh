# A/B of environment settings on one box: the default 3-stream C3 step alternated over REPS reps.
# usage (GPU box): bash tools/ab_env.sh "GSR_SPECULATE=0" "GSR_SPECULATE=1" ...
# TRAIN_STEPS=N adds the train.py call-site legs (immediate per-view backward) to every run.
set -o pipefail
mkdir -p gpurun_out/abenv
for rep in ${REPS:-1 2 3}; do
  k=0
  for e in "$@"; do
    k=$((k + 1))
    env $e timeout -k 10 200 python -u bench.py --steps ${STEPS:-200} ${BENCH_ARGS:-} \
      --call-site-steps 0 --train-steps ${TRAIN_STEPS:-0} --loss-steps 0 --densify-steps 0 --io-timesteps 0 --no-cpu-baseline \
      > gpurun_out/abenv/v$k.$rep.json 2> gpurun_out/abenv/v$k.$rep.err || { echo "$e failed"; tail -5 gpurun_out/abenv/v$k.$rep.err; exit 1; }
    python -c "
import json; d=json.loads([l for l in open('gpurun_out/abenv/v$k.$rep.json') if l.startswith('{')][0])
p=d['phase_ms_per_launch']; s=d['phase_ms_per_launch_solo']
print('$e rep=$rep', d['value'], d['median_ms_per_step'], d['value_mean'], d['step_ms_quartiles'], {k: (round(s[k]*1e3), round(p[k]*1e3)) for k in ('render_fwd','render_bwd','sum_records','gauss_bwd','bin_emit','bin_count') if k in s}, {k: (v['Msplats_per_s'], v['in_step_kernel_ms_per_launch']) for k, v in (d.get('train_call_site') or {}).items()})"
  done
done
