#!/bin/bash
# Round-4 GPU session script: each step under its own time limit; a fault / abort / timeout ends the
# script (no further GPU step), a plain test failure (rc 1) does not.
# usage (gpurun): bash tools/gpu_r04.sh "<pytest selection>" [bench args...]
set -u
mkdir -p gpurun_out
OUT=gpurun_out/r04
mkdir -p $OUT
fatal() { case $1 in 0|1|2) return 1;; *) return 0;; esac; }
SEL=${1:-}
shift || true
if [ -n "$SEL" ]; then
  timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread $SEL > $OUT/pytest.log 2>&1
  rc=$?; echo "pytest rc=$rc" | tee -a $OUT/status.txt
  tail -5 $OUT/pytest.log
  if fatal $rc; then echo "fatal pytest rc=$rc: stopping"; exit $rc; fi
fi
if [ "${1:-}" != "nobench" ]; then
  timeout -k 10 600 python -u bench.py "$@" > $OUT/bench.json 2> $OUT/bench.err
  rc=$?; echo "bench rc=$rc" | tee -a $OUT/status.txt
  tail -c 3000 $OUT/bench.err | tail -5
  if fatal $rc; then exit $rc; fi
fi
exit 0
