# Head-to-head on one box: round-1 tree (tools/ab/r01, built in place) vs the current tree with each
# tools/ab/libgsr_<v>.so variant, default 3-stream C3 step, alternated.  usage: bash tools/ab_r01.sh v1 v2 ...
set -o pipefail
mkdir -p gpurun_out/abr
for rep in $(seq 1 ${REPS:-2}); do
  for v in r01 "$@"; do
    if [ $v = r01 ]; then cmd="python -u tools/ab/r01/bench.py"; else cmd="env GSR_LIB=$(pwd)/tools/ab/libgsr_$v.so python -u bench.py"; fi
    timeout -k 10 200 $cmd --steps ${STEPS:-40} --call-site-steps 0 --loss-steps 0 --densify-steps 0 --io-timesteps 0 \
      --no-cpu-baseline ${BENCH_ARGS:-} > gpurun_out/abr/$v.$rep.json 2> gpurun_out/abr/$v.$rep.err || { echo "$v failed"; tail -5 gpurun_out/abr/$v.$rep.err; exit 1; }
    python -c "
import json; d=json.loads([l for l in open('gpurun_out/abr/$v.$rep.json') if l.startswith('{')][0])
print('$v rep=$rep value', d['value'], 'ms/step', d['ms_per_step'])"
  done
done
