#!/bin/bash
# full GPU suite, then the call-shape variants (one process each), then the headline bench
set -u
mkdir -p gpurun_out/r04
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > gpurun_out/r04/gpu_suite.log 2>&1
rc=$?; tail -3 gpurun_out/r04/gpu_suite.log; echo "suite rc=$rc"
case $rc in 0|1) ;; *) exit $rc;; esac
O=gpurun_out/r04/callshape.jsonl; : > $O
for v in "all_on --c2" "no_vs --no-view-streams" "none --no-async --no-view-streams" "all_on2"; do
  timeout -k 10 180 python -u tools/callshape_probe.py $v >> $O 2>> gpurun_out/r04/callshape.err
  rc=$?; case $rc in 0|1) ;; *) echo "fatal $rc"; exit $rc;; esac
done
cat $O
timeout -k 10 600 python -u bench.py > gpurun_out/r04/bench.json 2> gpurun_out/r04/bench.err
rc=$?; echo "bench rc=$rc"; case $rc in 0|1) ;; *) exit $rc;; esac
python3 -c "
import json; d=json.loads(open('gpurun_out/r04/bench.json').read().strip().splitlines()[-1])
print('value', d['value'], d['median_ms_per_step'], d['step_ms_quartiles']); print('unchanged', d['unchanged_call_site']); print('c2', d['c2']); print('host', d['host_ms_per_call']); print('train', {k: v['Msplats_per_s'] for k, v in d['train_call_site'].items()})"
