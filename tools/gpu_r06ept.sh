# Round 6: the exact re-walk (k_render_tsat) with several list entries per lane and round (GSR_TSAT_EPT):
# parity, the kernel's duration in a kernel trace of the inference leg, then alternated A/Bs.
set -o pipefail
O=gpurun_out/r06ept; mkdir -p $O
for v in ept4 ept8; do
  GSR_LIB=tools/ab/libgsr_$v.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_inference.py tests/test_headline_parity.py -m gpu -q --timeout 300 --timeout-method thread > $O/pytest_$v.log 2>&1 || { tail -20 $O/pytest_$v.log; exit 1; }
  echo "$v parity: $(tail -1 $O/pytest_$v.log)"
done
LEGS="--call-site-steps 0 --train-steps 0 --loss-steps 0 --densify-steps 0 --io-timesteps 0 --c2-steps 0 --no-cpu-baseline --unchanged-steps 0 --inference-steps 20 --steps 3 --warmup 1"
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for v in base ept2 ept4 ept8; do
  export GSR_LIB=tools/ab/libgsr_$v.so
  timeout -k 10 300 rocprofv3 --kernel-trace -f csv -d $O/prof_$v -o t -- python3 bench.py $LEGS > $O/prof_$v.log 2>&1 || { echo "prof $v failed"; tail -5 $O/prof_$v.log; exit 1; }
  python3 - $O/prof_$v/t_kernel_trace.csv $v <<'PY'
import csv, sys
rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r['Start_Timestamp']))
last = max(i for i, r in enumerate(rows) if 'gauss_bwd_multi' in r['Kernel_Name'])
def med(rr, k):
    v = sorted((int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3 for r in rr if k in r['Kernel_Name'])
    return (v[len(v) // 2], len(v)) if v else (None, 0)
print(sys.argv[2], 'step tsat', med(rows[:last], 'k_render_tsat'), 'inference tsat', med(rows[last + 1:], 'k_render_tsat'),
      'inference fwd', med(rows[last + 1:], 'k_render_fwd'))
PY
done
unset GSR_LIB
LEGS2="--call-site-steps 0 --train-steps 0 --loss-steps 0 --densify-steps 0 --io-timesteps 0 --c2-steps 0 --no-cpu-baseline --unchanged-steps 0 --inference-steps 40 --steps 3 --warmup 1"
for r in 1 2; do
  for v in base ept4 ept8; do
    GSR_LIB=tools/ab/libgsr_$v.so timeout -k 10 300 python -u bench.py $LEGS2 > $O/inf_$v$r.json 2> $O/inf_$v$r.err || { echo "$v failed"; tail -5 $O/inf_$v$r.err; exit 1; }
    python3 -c "
import json; d=json.loads(open('$O/inf_$v$r.json').read().strip().splitlines()[-1]); u=d['inference_call_site']
print('inference $v', u['Msplats_per_s'], u['median_ms_per_step'])"
  done
done
bash tools/lib_ab.sh $O 2 base ept4 ept8 || exit 1
