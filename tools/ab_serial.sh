# One-stream C3 step per tools/ab/libgsr_<v>.so variant, alternated, with per-phase times (us).
# usage (GPU box): bash tools/ab_serial.sh v1 v2 ...
set -o pipefail
mkdir -p gpurun_out/abs1
for rep in 1 2; do
  for v in "$@"; do
    GSR_LIB=$(pwd)/tools/ab/libgsr_$v.so timeout -k 10 200 python -u bench.py --streams 1 --steps 20 --call-site-steps 0 --loss-steps 0 --densify-steps 0 --io-timesteps 0 \
      --no-cpu-baseline ${BENCH_ARGS:-} > gpurun_out/abs1/$v.$rep.json 2> gpurun_out/abs1/$v.$rep.err || { echo "$v failed"; tail -5 gpurun_out/abs1/$v.$rep.err; exit 1; }
    python -c "
import json; d=json.loads([l for l in open('gpurun_out/abs1/$v.$rep.json') if l.startswith('{')][0])
print('$v rep=$rep value', d['value'], 'ms/step', d['ms_per_step'], {k: round(v*1e3) for k, v in d['phase_ms_per_launch'].items()})"
  done
done
