# Multi-view backward iteration: new tests first, then the whole GPU suite, then both step shapes.
set -o pipefail
out=gpurun_out/${1:-mv}; mkdir -p $out
timeout -k 10 300 python -u -m pytest tests/test_multiview.py -x -v --timeout 120 --timeout-method thread > $out/pytest_mv.log 2>&1 || { echo "mv tests failed"; tail -40 $out/pytest_mv.log; exit 1; }
tail -3 $out/pytest_mv.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $out/pytest.log 2>&1 || { echo "pytest failed"; tail -40 $out/pytest.log; exit 1; }
tail -2 $out/pytest.log
for shape in summed per-view; do
  timeout -k 10 300 python -u bench.py --step-shape $shape --call-site-steps 0 --loss-steps 0 --densify-steps 0 --io-timesteps 0 --no-cpu-baseline > $out/bench_$shape.json 2> $out/bench_$shape.err || { echo "bench $shape failed"; tail -20 $out/bench_$shape.err; exit 1; }
  python -c "
import json; d=json.loads([l for l in open('$out/bench_$shape.json') if l.startswith('{')][0])
print('$shape', 'value', d['value'], 'ms/step', d['ms_per_step'], 'dom', d['roofline']['kernel'], d['roofline']['avg_kernel_ms'])
print('phases', d['phase_ms_per_launch'])"
done
timeout -k 10 300 python -u bench.py --streams 1 --steps 10 --call-site-steps 0 --loss-steps 0 --densify-steps 0 --io-timesteps 0 --no-cpu-baseline > $out/bench1.json 2> $out/bench1.err || { echo "bench1 failed"; tail -20 $out/bench1.err; exit 1; }
python -c "
import json; d=json.loads([l for l in open('$out/bench1.json') if l.startswith('{')][0])
print('1-stream summed value', d['value'], 'ms/step', d['ms_per_step'])
print('1-stream phases', {k: round(v*1e3) for k, v in d['phase_ms_per_launch'].items()})"
