# Round 6: k_render_tsat block size (list entries per re-walk round): 64 / 128 (shipped) / 256, parity of
# the exact-saturation tests with each, then alternated A/B of the solo render_fwd phase.
set -o pipefail
O=gpurun_out/r06tsat; mkdir -p $O
for v in tsat64 tsat256; do
  GSR_LIB=tools/ab/libgsr_$v.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_headline_parity.py -m gpu -q --timeout 300 --timeout-method thread > $O/pytest_$v.log 2>&1 || { tail -20 $O/pytest_$v.log; exit 1; }
  echo "$v: $(tail -1 $O/pytest_$v.log)"
done
bash tools/lib_ab.sh $O 3 tsat128 tsat64 tsat256 || exit 1
