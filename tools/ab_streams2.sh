# Summed step with one submitting thread per stream: 2..5 streams, alternated twice.
set -o pipefail
mkdir -p gpurun_out/abst
for rep in 1 2; do
  for n in 3 4 5 2; do
    timeout -k 10 200 python -u bench.py --streams $n --steps 30 --call-site-steps 0 --loss-steps 0 --densify-steps 0 --io-timesteps 0 \
      --no-cpu-baseline > gpurun_out/abst/$n.$rep.json 2> gpurun_out/abst/$n.$rep.err || { echo "$n failed"; tail -5 gpurun_out/abst/$n.$rep.err; exit 1; }
    python -c "
import json; d=json.loads([l for l in open('gpurun_out/abst/$n.$rep.json') if l.startswith('{')][0])
print('streams=$n rep=$rep value', d['value'], 'ms/step', d['ms_per_step'])"
  done
done
