# Round-3 GPU pass: the whole -m gpu suite (stats for the flip allowances), then the bench lines.
set -o pipefail
tag=${1:-r03a}
mkdir -p gpurun_out/$tag
timeout -k 10 1200 python -u -m pytest tests -m gpu -v --timeout 600 --timeout-method thread > gpurun_out/$tag/pytest.log 2>&1
rc=$?
cp gpurun_out/parity_stats.json gpurun_out/$tag/ 2>/dev/null
echo "pytest rc $rc"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 400 python -u bench.py > gpurun_out/$tag/bench_c3.json 2> gpurun_out/$tag/bench_c3.err && \
timeout -k 10 300 python -u bench.py --config C2 --no-cpu-baseline > gpurun_out/$tag/bench_c2.json 2> gpurun_out/$tag/bench_c2.err && \
timeout -k 10 400 python -u bench.py --config C5 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/$tag/bench_c5.json 2> gpurun_out/$tag/bench_c5.err
echo "exit $?"
