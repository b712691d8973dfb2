# Round 6 final: the headline line of the shipped build in 4 fresh processes (run-to-run spread).
set -o pipefail
O=gpurun_out/r06spread; mkdir -p $O
LEGS="--call-site-steps 0 --train-steps 0 --loss-steps 0 --densify-steps 0 --io-timesteps 0 --c2-steps 0 --no-cpu-baseline --inference-steps 0 --unchanged-steps 0"
for r in 1 2 3 4; do
  timeout -k 10 300 python -u bench.py $LEGS > $O/b$r.json 2> $O/b$r.err || { echo "run $r failed"; tail -5 $O/b$r.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('$O/b$r.json').read().strip().splitlines()[-1])
print('run $r', d['value'], d['median_ms_per_step'], d['step_ms_quartiles'], 'solo fwd/bwd/gbwd', d['phase_ms_per_launch_solo']['render_fwd'], d['phase_ms_per_launch_solo']['render_bwd'], d['phase_ms_per_launch_solo']['gauss_bwd'])"
done
