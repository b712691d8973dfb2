set -o pipefail
mkdir -p gpurun_out/cfg
L="--no-cpu-baseline --call-site-steps 0 --inference-steps 0 --train-steps 0 --loss-steps 0 --densify-steps 0 --io-timesteps 0 --unchanged-steps 0 --c2-steps 0"
for c in C3M C4 C5; do
  timeout -k 10 300 python -u bench.py --config $c --steps 3 --warmup 1 $L > gpurun_out/cfg/$c.json 2> gpurun_out/cfg/$c.err || { echo "$c failed"; tail -5 gpurun_out/cfg/$c.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('gpurun_out/cfg/$c.json').read().strip().splitlines()[-1]); print('$c', d['value'], d['unit'], d['ms_per_step'], d['config'])"
done
