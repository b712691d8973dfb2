# Round 6: the long lists (n > 2048) blended by k_render_fwd_long (4-entry ILP walk) on a second stream --
# long-list parity tests, the suite, headline A/B against HEAD, C3M with both libraries and the per-wave
# trace of C3M's render.
set -o pipefail
O=gpurun_out/r06q; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "long_tile or segment_lengths" > $O/pytest_long.log 2>&1 || { tail -30 $O/pytest_long.log; exit 1; }
tail -2 $O/pytest_long.log
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -3 $O/pytest.log; cp gpurun_out/parity_stats.json $O/ 2>/dev/null
[ $rc -le 1 ] || exit $rc
bash tools/lib_ab.sh $O 2 def head || exit 1
R=$(pwd)
LEGS="--call-site-steps 0 --train-steps 0 --loss-steps 0 --densify-steps 0 --io-timesteps 0 --c2-steps 0 --no-cpu-baseline --inference-steps 0 --unchanged-steps 0"
for v in head def; do
  if [ $v = head ]; then export GSR_LIB=$R/tools/ab/libgsr_head.so; else unset GSR_LIB; fi
  timeout -k 10 300 python -u bench.py --config C3M $LEGS --steps 10 --warmup 3 > $O/c3m_$v.json 2> $O/c3m_$v.err || { echo "c3m $v failed"; tail -3 $O/c3m_$v.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('$O/c3m_$v.json').read().strip().splitlines()[-1]); s=d['phase_ms_per_launch_solo']
print('C3M $v', d['value'], d['median_ms_per_step'], 'solo fwd/bwd', s['render_fwd'], s['render_bwd'])"
done
unset GSR_LIB
GSR_TRACE_LIB=$R/tools/ab/libgsr_trace_head.so timeout -k 10 300 python -u tools/render_trace.py --config C3M --cams 0 > $O/trace_c3m_head.txt 2>&1 && grep "fwd\]" $O/trace_c3m_head.txt | cut -c1-300
timeout -k 10 300 python -u tools/render_trace.py --config C3M --cams 0 > $O/trace_c3m_def.txt 2>&1 && grep "fwd\]" $O/trace_c3m_def.txt | cut -c1-300
exit $rc
