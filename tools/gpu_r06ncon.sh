# Round 6: the T-saturation flag's drift window counted over the pixel's contributors (GSR_TSAT_NCON=1)
# instead of its list entries: parity, flagged pixels, the inference call site and the headline, alternated.
set -o pipefail
O=gpurun_out/r06ncon; mkdir -p $O
GSR_LIB=tools/ab/libgsr_ncon.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_inference.py tests/test_headline_parity.py -m gpu -q --timeout 300 --timeout-method thread > $O/pytest_ncon.log 2>&1 || { tail -20 $O/pytest_ncon.log; exit 1; }
echo "ncon parity: $(tail -1 $O/pytest_ncon.log)"
for v in base ncon; do
  GSR_LIB=tools/ab/libgsr_$v.so timeout -k 10 300 python -u tools/tsat_probe.py C3 1 > $O/probe_$v.log 2>&1 || { tail -5 $O/probe_$v.log; exit 1; }
  echo "$v $(tail -1 $O/probe_$v.log)"
done
LEGS="--call-site-steps 0 --train-steps 0 --loss-steps 0 --densify-steps 0 --io-timesteps 0 --c2-steps 0 --no-cpu-baseline --unchanged-steps 0 --inference-steps 40 --steps 3 --warmup 1"
for r in 1 2 3; do
  for v in base ncon; do
    GSR_LIB=tools/ab/libgsr_$v.so timeout -k 10 300 python -u bench.py $LEGS > $O/inf_$v$r.json 2> $O/inf_$v$r.err || { echo "$v failed"; tail -5 $O/inf_$v$r.err; exit 1; }
    python3 -c "
import json; d=json.loads(open('$O/inf_$v$r.json').read().strip().splitlines()[-1]); u=d['inference_call_site']
print('inference $v', u['Msplats_per_s'], u['median_ms_per_step'])"
  done
done
bash tools/lib_ab.sh $O 3 base ncon || exit 1
