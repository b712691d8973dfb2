#!/bin/bash
# A/B of the unchanged train.py call shape under the round-4 switches + a kernel trace of the default.
set -u
mkdir -p gpurun_out/r04
O=gpurun_out/r04/callshape.jsonl
: > $O
run() { timeout -k 10 180 "$@" >> $O 2> gpurun_out/r04/callshape.err; rc=$?; case $rc in 0|1) ;; *) echo "fatal rc=$rc"; exit $rc;; esac; }
run python -u tools/callshape_probe.py all_on --c2 --profile
run python -u tools/callshape_probe.py no_view_streams --no-view-streams --profile
run python -u tools/callshape_probe.py no_async --no-async --profile
GSR_ITEMS_AUX=0 run python -u tools/callshape_probe.py no_items_aux
GSR_ITEMS_AUX=0 run python -u tools/callshape_probe.py none --no-async --no-view-streams
run python -u tools/callshape_probe.py no_async_no_vs --no-async --no-view-streams --profile
run python -u tools/callshape_probe.py all_on_again
cat $O
bash tools/r04_headline_ab.sh || exit $?
R=$(pwd); T=$R/gpurun_out/r04/trace_unchanged
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$T" -- python3 "$R/tools/callshape_probe.py" traced --steps 20 > "$R/gpurun_out/r04/trace_unchanged.log" 2>&1 || { echo "trace failed"; exit 1; }
cd "$R"
python3 tools/stream_paths.py "$T" --frac 0.3 --gaps 30 > gpurun_out/r04/trace_unchanged_paths.txt 2>&1
head -60 gpurun_out/r04/trace_unchanged_paths.txt
