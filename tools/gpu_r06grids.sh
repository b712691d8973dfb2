# Round 6: launch grids of the two small exact-mode kernels -- k_render_bwd<true> (overflow tiles, 256
# blocks shipped) and k_render_tsat (4096 blocks shipped): fewer blocks wait less for dispatch inside the
# 3-stream step.  Parity of the variants, then alternated A/B.
set -o pipefail
O=gpurun_out/r06grids; mkdir -p $O
for v in exb32 tsb1024; do
  GSR_LIB=tools/ab/libgsr_$v.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -q --timeout 300 --timeout-method thread > $O/pytest_$v.log 2>&1 || { tail -20 $O/pytest_$v.log; exit 1; }
  echo "$v: $(tail -1 $O/pytest_$v.log)"
done
bash tools/lib_ab.sh $O 4 base exb32 tsb1024 || exit 1
