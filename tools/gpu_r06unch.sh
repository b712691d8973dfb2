# Round 6: the unchanged train.py call site (one thread, current stream) with blocking vs asynchronous
# forwards (GSR_ASYNC_FORWARD=1: no host wait for the pair count per view), alternated.
set -o pipefail
O=gpurun_out/r06unch; mkdir -p $O
LEGS="--call-site-steps 0 --train-steps 0 --loss-steps 0 --densify-steps 0 --io-timesteps 0 --c2-steps 0 --no-cpu-baseline --inference-steps 0 --unchanged-steps 40 --steps 5 --warmup 2"
for r in 1 2; do
  for v in block async; do
    if [ $v = async ]; then export GSR_ASYNC_FORWARD=1; else unset GSR_ASYNC_FORWARD; fi
    timeout -k 10 300 python -u bench.py $LEGS > $O/$v$r.json 2> $O/$v$r.err || { echo "$v failed"; tail -5 $O/$v$r.err; exit 1; }
    python3 -c "
import json; d=json.loads(open('$O/$v$r.json').read().strip().splitlines()[-1]); u=d['unchanged_call_site']
print('$v', u['Msplats_per_s'], u['median_ms_per_step'], 'host', u.get('host_ms_per_step_median'))"
  done
done
