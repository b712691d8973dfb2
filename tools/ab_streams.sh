# Pipelined C3 step at several stream counts, alternated.  usage (GPU box): bash tools/ab_streams.sh 2 3 4 5
set -o pipefail
mkdir -p gpurun_out/abs
for rep in 1 2; do
  for n in "$@"; do
    timeout -k 10 200 python -u bench.py --steps 60 --streams $n --call-site-steps 0 --loss-steps 0 --densify-steps 0 --io-timesteps 0 \
      --no-cpu-baseline ${BENCH_ARGS:-} > gpurun_out/abs/s$n.$rep.json 2> gpurun_out/abs/s$n.$rep.err || { echo "s$n failed"; tail -5 gpurun_out/abs/s$n.$rep.err; exit 1; }
    python -c "
import json; d=json.loads([l for l in open('gpurun_out/abs/s$n.$rep.json') if l.startswith('{')][0])
print('streams $n rep=$rep value', d['value'], 'ms/step', d['ms_per_step'], 'host', d.get('host_ms_per_call'))"
  done
done
