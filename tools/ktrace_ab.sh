# rocprofv3 kernel traces of the default (3-stream) C3 bench step for the round-1 tree and the current
# tree, each followed by tools/concurrency.py over the timed region.  usage (GPU box): bash tools/ktrace_ab.sh
set -u
R=$(pwd); O=$R/gpurun_out/ktab; mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
for v in r01 cur; do
  if [ $v = r01 ]; then B=$R/tools/ab/r01/bench.py; else B=$R/bench.py; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$O/$v" -- \
      python3 "$B" --no-cpu-baseline --call-site-steps 0 --loss-steps 0 --densify-steps 0 --io-timesteps 0 > "$O/$v.log" 2>&1 || { echo "$v trace failed"; exit 1; }
  echo "== $v"; grep '^{' "$O/$v.log" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])"
  python3 $R/tools/concurrency.py "$O/$v" --from-launch k_render_bwd 40 140
done
