# Summed-step submission A/B: serial vs one host thread per stream, 3 and 5 streams (alternated twice).
set -o pipefail
mkdir -p gpurun_out/absub
for rep in 1 2; do
  for cfg in "serial 3" "threads 3" "serial 5" "threads 5" "serial 2"; do
    set -- $cfg
    timeout -k 10 200 python -u bench.py --submit $1 --streams $2 --steps 30 --call-site-steps 0 --loss-steps 0 --densify-steps 0 --io-timesteps 0 \
      --no-cpu-baseline > gpurun_out/absub/$1.$2.$rep.json 2> gpurun_out/absub/$1.$2.$rep.err || { echo "$cfg failed"; tail -5 gpurun_out/absub/$1.$2.$rep.err; exit 1; }
    python -c "
import json; d=json.loads([l for l in open('gpurun_out/absub/$1.$2.$rep.json') if l.startswith('{')][0])
print('$1 streams=$2 rep=$rep value', d['value'], 'ms/step', d['ms_per_step'], 'host', d['host_ms_per_call'])"
  done
done
