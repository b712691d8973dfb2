#!/bin/bash
# unchanged call shape: library view streams (count, helper thread) vs none, alternated
set -u
mkdir -p gpurun_out/r04
O=gpurun_out/r04/vsn.jsonl; : > $O
for r in 1 2; do
  timeout -k 10 180 python -u tools/callshape_probe.py none --no-async --no-view-streams --steps 40 >> $O 2>> gpurun_out/r04/vsn.err || exit 1
  GSR_VIEW_STREAMS_N=1 GSR_VIEW_HELPER=0 timeout -k 10 180 python -u tools/callshape_probe.py vs1_nohelper --no-async --steps 40 >> $O 2>> gpurun_out/r04/vsn.err || exit 1
  GSR_VIEW_STREAMS_N=1 timeout -k 10 180 python -u tools/callshape_probe.py vs1_helper --no-async --steps 40 >> $O 2>> gpurun_out/r04/vsn.err || exit 1
  GSR_VIEW_STREAMS_N=2 GSR_VIEW_HELPER=0 timeout -k 10 180 python -u tools/callshape_probe.py vs2_nohelper --no-async --steps 40 >> $O 2>> gpurun_out/r04/vsn.err || exit 1
done
python3 -c "
import json
for l in open('$O'):
    d=json.loads(l); u=d['unchanged']; print(d['name'], u['Msplats_per_s'], u['median_ms_per_step'], u['host_ms_per_step_median'])"
