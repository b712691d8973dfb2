# Default C3 bench under several argument sets, alternated.  usage (GPU box):
#   bash tools/ab_args.sh "--submit serial" "--submit threads" ...
set -o pipefail
mkdir -p gpurun_out/aba
for rep in $(seq 1 ${REPS:-2}); do
  i=0
  for a in "$@"; do
    i=$((i+1))
    timeout -k 10 200 python -u bench.py --steps ${STEPS:-40} --train-steps 0 --call-site-steps 0 --loss-steps 0 --densify-steps 0 --io-timesteps 0 \
      --no-cpu-baseline $a > gpurun_out/aba/$i.$rep.json 2> gpurun_out/aba/$i.$rep.err || { echo "[$a] failed"; tail -5 gpurun_out/aba/$i.$rep.err; exit 1; }
    python -c "
import json; d=json.loads([l for l in open('gpurun_out/aba/$i.$rep.json') if l.startswith('{')][0])
print('[$a] rep=$rep value', d['value'], 'ms/step', d['ms_per_step'], 'host', d.get('host_ms_per_call'))"
  done
done
