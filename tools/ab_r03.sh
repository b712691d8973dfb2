# A/B of libgsr variants (tools/ab/libgsr_<v>.so): a parity subset per variant (GSR_LIB), then the
# default 3-stream C3 step alternated over REPS reps with solo + in-step phase times.
# usage (GPU box): bash tools/ab_r03.sh v1 v2 ...
set -o pipefail
mkdir -p gpurun_out/abr3
for v in "$@"; do
  GSR_LIB=$(pwd)/tools/ab/libgsr_$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_multiview.py \
    -m gpu -x -q --timeout 200 --timeout-method thread -k "${PARITY_K:-c1 or sh3 or C3_yaw0 or long_tile or deferred_equals}" \
    > gpurun_out/abr3/$v.pytest.log 2>&1 || { echo "$v parity failed"; tail -30 gpurun_out/abr3/$v.pytest.log; exit 1; }
  echo "$v parity ok: $(tail -1 gpurun_out/abr3/$v.pytest.log)"
done
for rep in ${REPS:-1 2 3}; do
  for v in "$@"; do
    GSR_LIB=$(pwd)/tools/ab/libgsr_$v.so timeout -k 10 200 python -u bench.py --steps ${STEPS:-200} ${BENCH_ARGS:-} \
      --call-site-steps 0 --train-steps 0 --loss-steps 0 --densify-steps 0 --io-timesteps 0 --no-cpu-baseline \
      > gpurun_out/abr3/$v.$rep.json 2> gpurun_out/abr3/$v.$rep.err || { echo "$v failed"; tail -5 gpurun_out/abr3/$v.$rep.err; exit 1; }
    python -c "
import json; d=json.loads([l for l in open('gpurun_out/abr3/$v.$rep.json') if l.startswith('{')][0])
p=d['phase_ms_per_launch']; s=d['phase_ms_per_launch_solo']
print('$v rep=$rep', d['value'], d['median_ms_per_step'], d['value_mean'], {k: (round(s[k]*1e3), round(p[k]*1e3)) for k in '${PHASES:-render_fwd render_bwd gauss_bwd bin_emit}'.split()})"
  done
done
