# Round 6: where the per-tile depth sort runs -- inside k_render_fwd for lists up to GSR_FWD_SORT_CAP
# (1024 shipped), the rest in k_tile_sort (one 512-thread block per list) -- parity with 0 and 256, then
# alternated A/B of the solo phases and the headline.
set -o pipefail
O=gpurun_out/r06sortcap; mkdir -p $O
for v in sc0 sc256; do
  GSR_LIB=tools/ab/libgsr_$v.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -q --timeout 300 --timeout-method thread > $O/pytest_$v.log 2>&1 || { tail -20 $O/pytest_$v.log; exit 1; }
  echo "$v: $(tail -1 $O/pytest_$v.log)"
done
bash tools/lib_ab.sh $O 3 sc1024 sc0 sc256 || exit 1
