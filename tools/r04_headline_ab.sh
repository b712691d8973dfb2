#!/bin/bash
# Headline step A/B under the round-4 switches (alternated reps, one process each).
set -u
mkdir -p gpurun_out/r04
O=gpurun_out/r04/headline_ab.txt
: > $O
B="--steps 100 --warmup 10 --no-cpu-baseline --probe-steps 0 --call-site-steps 0 --train-steps 0 --loss-steps 0 --densify-steps 0 --io-timesteps 0 --unchanged-steps 0 --c2-steps 0"
one() {
  tag=$1; shift
  env "$@" timeout -k 10 120 python -u bench.py $B > gpurun_out/r04/h.json 2> gpurun_out/r04/h.err
  rc=$?; case $rc in 0|1) ;; *) echo "fatal rc=$rc"; exit $rc;; esac
  python3 -c "import json,sys; d=json.loads(open('gpurun_out/r04/h.json').read().strip().splitlines()[-1]); print('$tag', d['value'], d['median_ms_per_step'], d['step_ms_quartiles'], d['host_ms_per_call'])" >> $O
}
for rep in 1 2; do
  one default GSR_X=1
  one no_items_aux GSR_ITEMS_AUX=0
  one no_async GSR_ASYNC_FORWARD=0
  one neither GSR_ITEMS_AUX=0 GSR_ASYNC_FORWARD=0
done
cat $O
