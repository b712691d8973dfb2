# A/B of GPU_MAX_HW_QUEUES (hardware queues per process) x view streams, default C3 step, alternated.
set -o pipefail
mkdir -p gpurun_out/abq
for rep in 1 2 3; do
  for cfg in "4 3" "8 3" "8 4" "8 5"; do
    set -- $cfg
    GPU_MAX_HW_QUEUES=$1 timeout -k 10 200 python -u bench.py --steps 100 --streams $2 --train-steps 0 --call-site-steps 0 --loss-steps 0 --densify-steps 0 --io-timesteps 0 --no-cpu-baseline > gpurun_out/abq/q$1s$2.$rep.json 2> gpurun_out/abq/q$1s$2.$rep.err || { echo "q$1 s$2 failed"; tail -3 gpurun_out/abq/q$1s$2.$rep.err; exit 1; }
    python -c "
import json; d=json.loads([l for l in open('gpurun_out/abq/q$1s$2.$rep.json') if l.startswith('{')][0])
print('queues $1 streams $2 rep $rep', d['value'], d['median_ms_per_step'])"
  done
done
