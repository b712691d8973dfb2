# Round 6: packed-chain saturation re-walk (v3) -- suite, A/B against the pre-re-walk library, its kernel
# time (trace), and the clustered C3M config (long lists) with both libraries.
set -o pipefail
O=gpurun_out/r06i; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -3 $O/pytest.log; cp gpurun_out/parity_stats.json $O/ 2>/dev/null
[ $rc -le 1 ] || exit $rc
bash tools/lib_ab.sh $O 3 base def || exit 1
R=$(pwd)
LEGS="--call-site-steps 0 --train-steps 0 --loss-steps 0 --densify-steps 0 --io-timesteps 0 --c2-steps 0 --no-cpu-baseline --inference-steps 0 --unchanged-steps 0"
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/trace -- python3 $R/bench.py $LEGS --steps 20 --warmup 5 > $R/$O/trace.log 2>&1) || { echo "trace failed"; exit 1; }
python3 tools/rocprof_summary.py trace $O/trace > $O/trace_summary.txt; head -16 $O/trace_summary.txt
for v in base def; do
  if [ $v = base ]; then export GSR_LIB=$R/tools/ab/libgsr_base.so; else unset GSR_LIB; fi
  timeout -k 10 300 python -u bench.py --config C3M $LEGS --steps 10 --warmup 3 > $O/c3m_$v.json 2> $O/c3m_$v.err || { echo "c3m $v failed"; tail -3 $O/c3m_$v.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('$O/c3m_$v.json').read().strip().splitlines()[-1]); s=d['phase_ms_per_launch_solo']
print('C3M $v', d['value'], d['median_ms_per_step'], 'solo fwd/bwd', s['render_fwd'], s['render_bwd'])"
done
timeout -k 10 300 python -u tools/t_drift.py C3 1 > $O/drift_C3.log 2>&1 && grep -v amdgpu $O/drift_C3.log | head -3
exit $rc
