#!/bin/bash
# unchanged call shape: number of library view streams (GSR_VIEW_STREAMS_N), async on/off
set -u
mkdir -p gpurun_out/r04
O=gpurun_out/r04/vsn.jsonl; : > $O
for n in 1 2 3 1; do
  GSR_VIEW_STREAMS_N=$n timeout -k 10 180 python -u tools/callshape_probe.py vs$n --steps 40 >> $O 2>> gpurun_out/r04/vsn.err
  rc=$?; case $rc in 0|1) ;; *) echo "fatal $rc"; exit $rc;; esac
done
GSR_VIEW_STREAMS_N=1 timeout -k 10 180 python -u tools/callshape_probe.py vs1_noasync --no-async --steps 40 >> $O 2>> gpurun_out/r04/vsn.err
timeout -k 10 180 python -u tools/callshape_probe.py none --no-async --no-view-streams --steps 40 >> $O 2>> gpurun_out/r04/vsn.err
cat $O
