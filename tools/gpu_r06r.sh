# Round 6: k_render_fwd_long with two-stage record prefetch + high-priority side stream -- long-list parity
# tests, C3M with this library, the per-wave trace of C3M's render.
set -o pipefail
O=gpurun_out/r06r; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "long_tile or segment_lengths" > $O/pytest_long.log 2>&1 || { tail -30 $O/pytest_long.log; exit 1; }
tail -1 $O/pytest_long.log
LEGS="--call-site-steps 0 --train-steps 0 --loss-steps 0 --densify-steps 0 --io-timesteps 0 --c2-steps 0 --no-cpu-baseline --inference-steps 0 --unchanged-steps 0"
timeout -k 10 300 python -u bench.py --config C3M $LEGS --steps 10 --warmup 3 > $O/c3m_def.json 2> $O/c3m_def.err || { echo "c3m failed"; tail -3 $O/c3m_def.err; exit 1; }
python3 -c "
import json; d=json.loads(open('$O/c3m_def.json').read().strip().splitlines()[-1]); s=d['phase_ms_per_launch_solo']
print('C3M def', d['value'], d['median_ms_per_step'], 'solo fwd/bwd', s['render_fwd'], s['render_bwd'])"
timeout -k 10 300 python -u tools/render_trace.py --config C3M --cams 0 > $O/trace_c3m_def.txt 2>&1 && grep "fwd" $O/trace_c3m_def.txt | cut -c1-330
