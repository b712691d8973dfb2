# Round 6 final: the default bench line (as the driver runs it), then C3M.
set -o pipefail
O=gpurun_out/r06bench; mkdir -p $O
timeout -k 10 1000 python -u bench.py > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail -20 $O/bench.err; exit 1; }
tail -1 $O/bench.json
LEGS="--call-site-steps 0 --train-steps 0 --loss-steps 0 --densify-steps 0 --io-timesteps 0 --c2-steps 0 --no-cpu-baseline --inference-steps 0 --unchanged-steps 0"
timeout -k 10 300 python -u bench.py --config C3M $LEGS --steps 10 --warmup 3 > $O/c3m.json 2> $O/c3m.err || { echo "c3m failed"; tail -3 $O/c3m.err; exit 1; }
python3 -c "
import json; d=json.loads(open('$O/c3m.json').read().strip().splitlines()[-1]); s=d['phase_ms_per_launch_solo']
print('C3M', d['value'], d['median_ms_per_step'], 'solo fwd/bwd', s['render_fwd'], s['render_bwd'])"
