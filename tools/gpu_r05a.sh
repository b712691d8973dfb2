set -o pipefail
mkdir -p gpurun_out/r05a
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r05a/pytest.log 2>&1; rc=$?
tail -5 gpurun_out/r05a/pytest.log; cp gpurun_out/parity_stats.json gpurun_out/r05a/ 2>/dev/null
[ $rc -le 1 ] || exit $rc
bash tools/lib_ab.sh gpurun_out/r05a 2 r04 def || exit 1
bash tools/pmc_lib.sh gpurun_out/r05a r04 && bash tools/pmc_lib.sh gpurun_out/r05a def
