# Round 6: re-walk kernel with packed records + long-list batch skip -- suite, probes, A/Bs.
set -o pipefail
O=gpurun_out/r06l; mkdir -p $O
R=$(pwd)
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -3 $O/pytest.log; cp gpurun_out/parity_stats.json $O/ 2>/dev/null
[ $rc -le 1 ] || exit $rc
for c in C3 C3M; do
  (cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/probe_$c -- python3 $R/tools/tsat_probe.py $c 3 > $R/$O/probe_$c.log 2>&1) || { echo "probe $c failed"; tail -5 $O/probe_$c.log; exit 1; }
  grep -v "amdgpu\|^W20\|^E20" $O/probe_$c.log
  python3 tools/rocprof_summary.py trace $O/probe_$c | grep -E "render|tsat|long_cull" | head -6
done
bash tools/lib_ab.sh $O 3 base def || exit 1
LEGS="--call-site-steps 0 --train-steps 0 --loss-steps 0 --densify-steps 0 --io-timesteps 0 --c2-steps 0 --no-cpu-baseline --inference-steps 0 --unchanged-steps 0"
for r in 1 2; do
for v in nolong def; do
  if [ $v = nolong ]; then export GSR_LIB=$R/tools/ab/libgsr_nolong.so; else unset GSR_LIB; fi
  timeout -k 10 300 python -u bench.py --config C3M $LEGS --steps 10 --warmup 3 > $O/c3m_$v$r.json 2> $O/c3m_$v$r.err || { echo "c3m $v failed"; tail -3 $O/c3m_$v$r.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('$O/c3m_$v$r.json').read().strip().splitlines()[-1]); s=d['phase_ms_per_launch_solo']
print('C3M $v', d['value'], d['median_ms_per_step'], 'solo fwd/bwd/sort', s['render_fwd'], s['render_bwd'], s['tile_sort'])"
done
done
unset GSR_LIB
exit $rc
