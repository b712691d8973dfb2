set -o pipefail
tag=${1:-r02a}
mkdir -p gpurun_out/$tag
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/$tag/pytest.log 2>&1 && \
cp gpurun_out/parity_stats.json gpurun_out/$tag/ && \
timeout -k 10 300 python -u bench.py > gpurun_out/$tag/bench_c3.json 2> gpurun_out/$tag/bench_c3.err && \
timeout -k 10 300 python -u bench.py --config C4 --steps 5 --warmup 2 > gpurun_out/$tag/bench_c4.json 2> gpurun_out/$tag/bench_c4.err && \
timeout -k 10 300 python -u bench.py --config C5 --steps 10 --warmup 3 > gpurun_out/$tag/bench_c5.json 2> gpurun_out/$tag/bench_c5.err && \
timeout -k 10 300 python -u bench.py --gpus 2 --backend gloo --config C4 --steps 3 --warmup 1 > gpurun_out/$tag/bench_c4_gloo2.json 2> gpurun_out/$tag/bench_c4_gloo2.err
echo "exit $?"
