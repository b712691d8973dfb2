# Round 6 structural render_bwd variant: 8x8 backward quarters (GSR_BWD_Q8=1) -- parity
# with zero allowances, repeatability, alternated A/B against the default 16x4 strips, SQ counters.
# usage: bash tools/gpu_r06f.sh
set -o pipefail
O=gpurun_out/r06f; mkdir -p $O
GSR_BWD_Q8=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_headline_parity.py tests/test_repeatability.py tests/test_multiview.py -m gpu -q -x --timeout 300 --timeout-method thread > $O/pytest_q8.log 2>&1; rc=$?
tail -4 $O/pytest_q8.log
[ $rc -le 1 ] || exit $rc
LEGS="--call-site-steps 0 --train-steps 0 --loss-steps 0 --densify-steps 0 --io-timesteps 0 --c2-steps 0 --no-cpu-baseline --inference-steps 0 --unchanged-steps 0"
for r in 1 2 3; do
  for v in def q8; do
    if [ $v = q8 ]; then export GSR_BWD_Q8=1; else unset GSR_BWD_Q8; fi
    timeout -k 10 300 python -u bench.py $LEGS > $O/ab_$v$r.json 2> $O/ab_$v$r.err || { echo "bench $v failed"; exit 1; }
    python3 -c "
import json; d=json.loads(open('$O/ab_$v$r.json').read().strip().splitlines()[-1]); s=d['phase_ms_per_launch_solo']
print('$v', d['value'], d['median_ms_per_step'], 'solo fwd/bwd', s['render_fwd'], s['render_bwd'])"
  done
done
unset GSR_BWD_Q8
R=$(pwd)
for v in def q8; do
  if [ $v = q8 ]; then export GSR_BWD_Q8=1; else unset GSR_BWD_Q8; fi
  mkdir -p $O/pmc_$v
  (cd /tmp && export TMPDIR=/tmp && timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU_TRANS_F32 \
    --kernel-include-regex "render_bwd" --kernel-trace --output-format csv -d $R/$O/pmc_$v -- \
    python3 $R/bench.py --no-cpu-baseline --streams 1 --steps 6 --warmup 2 --probe-steps 1 $LEGS > $R/$O/pmc_$v/log 2>&1) || { echo "pmc $v failed"; exit 1; }
  python3 tools/pmc_table.py $O/pmc_$v 2>/dev/null | head -5 || true
done
unset GSR_BWD_Q8
python3 tools/rocprof_summary.py sq $O/pmc_def > $O/sq_def.txt; python3 tools/rocprof_summary.py sq $O/pmc_q8 > $O/sq_q8.txt
grep render_bwd $O/sq_def.txt $O/sq_q8.txt | cut -c1-600
