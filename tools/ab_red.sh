# Reduction-stage variants: stream-determinism test (bitwise 1 vs n streams) + parity on each, then A/B.
set -o pipefail
for v in red2 red1; do
  GSR_LIB=$(pwd)/tools/ab/libgsr_$v.so timeout -k 10 300 python -u -m pytest tests/test_streams.py tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -k "bitwise or forward_backward_parity or baseline_size_parity" > gpurun_out/red_$v.log 2>&1; echo "$v tests rc=$?"; tail -2 gpurun_out/red_$v.log
done
bash tools/ab_serial.sh red3 red2 red1
