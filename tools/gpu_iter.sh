# One GPU iteration: parity tests, a short bench, a per-wave trace of the render kernels.
# usage: bash tools/gpu_iter.sh <tag> [pytest -k expression]
set -o pipefail
tag=${1:-iter}; sel=${2:-}
out=gpurun_out/$tag; mkdir -p $out
if [ -n "$sel" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "$sel" > $out/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $out/pytest.log; exit 1; }
else
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $out/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $out/pytest.log; exit 1; }
fi
tail -2 $out/pytest.log
timeout -k 10 300 python -u bench.py --call-site-steps 0 --loss-steps 0 --densify-steps 0 --io-timesteps 0 --no-cpu-baseline > $out/bench.json 2> $out/bench.err || { echo "bench failed"; tail -20 $out/bench.err; exit 1; }
python -c "
import json; d=json.loads([l for l in open('$out/bench.json') if l.startswith('{')][0])
print('value', d['value'], 'ms/step', d['ms_per_step'], 'dom', d['roofline']['kernel'], d['roofline']['avg_kernel_ms'])
print('phases', d['phase_ms_per_launch'])"
timeout -k 10 300 python -u bench.py --streams 1 --steps 10 --call-site-steps 0 --loss-steps 0 --densify-steps 0 --io-timesteps 0 --no-cpu-baseline > $out/bench1.json 2> $out/bench1.err || { echo "bench1 failed"; tail -20 $out/bench1.err; exit 1; }
python -c "
import json; d=json.loads([l for l in open('$out/bench1.json') if l.startswith('{')][0])
print('1-stream value', d['value'], 'ms/step', d['ms_per_step'])
print('1-stream phases', {k: round(v*1e3) for k, v in d['phase_ms_per_launch'].items()})"
if [ -f tools/libgsr_trace.so ]; then
  timeout -k 10 300 python tools/render_trace.py --cams 0,9,13 > $out/trace.txt 2>&1 && grep -v amdgpu.ids $out/trace.txt | grep "fwd\]\|bwd\]" | cut -c1-400
fi
exit 0
