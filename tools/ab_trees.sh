# Head-to-head of whole trees on one box: tools/ab/<tree>/bench.py (each tree built in place), default
# 3-stream C3 step, alternated.  usage (GPU box): bash tools/ab_trees.sh r01 t_abc ...   ("." = this tree)
set -o pipefail
mkdir -p gpurun_out/abt
unset GSR_LIB
for rep in 1 2 3; do
  for v in "$@"; do
    if [ "$v" = . ]; then b=bench.py; n=cur; else b=tools/ab/$v/bench.py; n=$v; fi
    timeout -k 10 200 python -u $b --steps 60 --call-site-steps 0 --loss-steps 0 --densify-steps 0 --io-timesteps 0 \
      --no-cpu-baseline ${BENCH_ARGS:-} > gpurun_out/abt/$n.$rep.json 2> gpurun_out/abt/$n.$rep.err || { echo "$n failed"; tail -5 gpurun_out/abt/$n.$rep.err; exit 1; }
    python -c "
import json; d=json.loads([l for l in open('gpurun_out/abt/$n.$rep.json') if l.startswith('{')][0])
print('$n rep=$rep value', d['value'], 'ms/step', d['ms_per_step'])"
  done
done
