# Round evidence on one box: the whole -m gpu suite, the default bench line, then the rocprofv3
# trace + HBM + SQ passes (tools/profile_round.sh).  usage (GPU box): bash tools/gpu_full.sh <tag>
set -o pipefail
tag=${1:-r03}
mkdir -p gpurun_out/$tag
timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/$tag/pytest.log 2>&1
rc=$?
cp gpurun_out/parity_stats.json gpurun_out/$tag/ 2>/dev/null
echo "pytest rc $rc: $(tail -1 gpurun_out/$tag/pytest.log)"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 400 python -u bench.py > gpurun_out/$tag/bench.json 2> gpurun_out/$tag/bench.err || { echo "bench failed"; tail -5 gpurun_out/$tag/bench.err; exit 3; }
echo "bench: $(grep -o '"value": [0-9.]*' gpurun_out/$tag/bench.json | head -1)"
[ -n "${NO_PROFILE:-}" ] && exit 0
bash tools/profile_round.sh $tag
