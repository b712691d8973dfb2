set -o pipefail
O=gpurun_out/r05c; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_inference.py -m gpu -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -3 $O/pytest.log
[ $rc -le 1 ] || exit $rc
bash tools/lib_ab.sh $O 2 r04tree def || exit 1
bash tools/pmc_lib.sh $O r04tree lds && bash tools/pmc_lib.sh $O def lds && bash tools/pmc_lib.sh $O def sq
