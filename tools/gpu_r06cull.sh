# Round 6: the long lists' quarter cull done ahead over the whole chip
# (k_long_cull / k_long_compact), the render staging only the compacted entries -- long-list parity tests,
# the suite, C3M against the previous build, the per-wave trace of C3M's render, the headline A/B.
set -o pipefail
O=gpurun_out/r06cull; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "long_tile or segment_lengths" > $O/pytest_long.log 2>&1 || { tail -40 $O/pytest_long.log; exit 1; }
tail -1 $O/pytest_long.log
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -3 $O/pytest.log; cp gpurun_out/parity_stats.json $O/ 2>/dev/null
[ $rc -le 1 ] || exit $rc
LEGS="--call-site-steps 0 --train-steps 0 --loss-steps 0 --densify-steps 0 --io-timesteps 0 --c2-steps 0 --no-cpu-baseline --inference-steps 0 --unchanged-steps 0"
for v in def prev def prev; do
  if [ $v = prev ]; then export GSR_LIB=$(pwd)/tools/ab/libgsr_prev.so; else unset GSR_LIB; fi
  timeout -k 10 300 python -u bench.py --config C3M $LEGS --steps 10 --warmup 3 > $O/c3m_$v.json 2> $O/c3m_$v.err || { echo "c3m $v failed"; tail -3 $O/c3m_$v.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('$O/c3m_$v.json').read().strip().splitlines()[-1]); s=d['phase_ms_per_launch_solo']
print('C3M $v', d['value'], d['median_ms_per_step'], 'solo fwd/bwd', s['render_fwd'], s['render_bwd'])"
done
unset GSR_LIB
timeout -k 10 300 python -u tools/render_trace.py --config C3M --cams 0 > $O/trace_c3m.txt 2>&1 && grep "fwd\]" $O/trace_c3m.txt | cut -c1-230 && cp gpurun_out/trace_fwd_cam0.npy $O/trace_fwd.npy
GSR_TRACE_LIB=$(pwd)/tools/ab/libgsr_trace_prev.so timeout -k 10 300 python -u tools/render_trace.py --config C3M --cams 0 > $O/trace_c3m_prev.txt 2>&1 && grep "fwd\]" $O/trace_c3m_prev.txt | cut -c1-230
bash tools/lib_ab.sh $O 2 def prev || exit 1
exit $rc
