# Round 6: the inference call site (train.py's no_grad 5-camera renders, one thread, current stream)
# with the exact-threshold mode on (default) vs off, alternated; then one kernel trace of the default.
set -o pipefail
O=gpurun_out/r06inf; mkdir -p $O
LEGS="--call-site-steps 0 --train-steps 0 --loss-steps 0 --densify-steps 0 --io-timesteps 0 --c2-steps 0 --no-cpu-baseline --unchanged-steps 0 --inference-steps 40 --steps 3 --warmup 1"
for r in 1 2 3; do
  for v in exact fast; do
    if [ $v = fast ]; then export GSR_EXACT_THRESHOLDS=0; else unset GSR_EXACT_THRESHOLDS; fi
    timeout -k 10 300 python -u bench.py $LEGS > $O/$v$r.json 2> $O/$v$r.err || { echo "$v failed"; tail -5 $O/$v$r.err; exit 1; }
    python3 -c "
import json; d=json.loads(open('$O/$v$r.json').read().strip().splitlines()[-1]); u=d['inference_call_site']
print('$v', u['Msplats_per_s'], u['median_ms_per_step'], 'host', u.get('host_ms_per_step_median'))"
  done
done
unset GSR_EXACT_THRESHOLDS
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $O/prof -o inf -- python3 bench.py $LEGS > $O/prof.log 2>&1 && echo prof ok
