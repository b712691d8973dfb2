#!/bin/bash
# the default bench line only (plus its solo phase times)
set -u
mkdir -p gpurun_out/r04
timeout -k 10 600 python -u bench.py "$@" > gpurun_out/r04/bench.json 2> gpurun_out/r04/bench.err
rc=$?; echo "bench rc=$rc"; case $rc in 0|1) ;; *) exit $rc;; esac
python3 -c "
import json; d=json.loads(open('gpurun_out/r04/bench.json').read().strip().splitlines()[-1])
print('value', d['value'], d['median_ms_per_step'], d['step_ms_quartiles']); print('unchanged', {k: d['unchanged_call_site'][k] for k in ('Msplats_per_s','median_ms_per_step','host_ms_per_step_median')}); print('c2', {k: d['c2'][k] for k in ('Msplats_per_s','median_ms_per_step','host_ms_per_step_median','step_ms_quartiles')}); print('train', {k: v['Msplats_per_s'] for k, v in d['train_call_site'].items()})
print('solo', d.get('phase_ms_per_launch_solo')); print('step', d.get('phase_ms_per_launch'))"
