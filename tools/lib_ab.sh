#!/bin/bash
# A/B library builds on the bench (headline + solo phases), alternated on one box.
# usage: bash tools/lib_ab.sh OUTDIR REPS NAME...   (NAME = def -> the in-tree libgsr.so; NAMEtree -> the whole
# exported tree tools/ab/NAMEtree (its own bench.py, package and libraries); fast -> the in-tree library with
# the exact-threshold mode off; else tools/ab/libgsr_NAME.so)
set -u
O=$1; N=$2; shift 2
mkdir -p "$O"
LEGS="--call-site-steps 0 --train-steps 0 --loss-steps 0 --densify-steps 0 --io-timesteps 0 --c2-steps 0 --no-cpu-baseline"
for r in $(seq "$N"); do
  for v in "$@"; do
    case "$v" in
      def) GSR_LIB=animating-gaussian-splats_amd/diff_gaussian_rasterization/libgsr.so timeout -k 10 300 python -u bench.py $LEGS --inference-steps 0 > "$O/lab_$v$r.json" 2> "$O/lab_$v$r.err" ;;
      *_fast) GSR_EXACT_THRESHOLDS=0 GSR_LIB=tools/ab/libgsr_${v%_fast}.so timeout -k 10 300 python -u bench.py $LEGS --inference-steps 0 > "$O/lab_$v$r.json" 2> "$O/lab_$v$r.err" ;;
      fast) GSR_EXACT_THRESHOLDS=0 timeout -k 10 300 python -u bench.py $LEGS --inference-steps 0 > "$O/lab_$v$r.json" 2> "$O/lab_$v$r.err" ;;
      *tree) timeout -k 10 300 python -u tools/ab/$v/bench.py $LEGS > "$O/lab_$v$r.json" 2> "$O/lab_$v$r.err" ;;
      *) GSR_LIB=tools/ab/libgsr_$v.so timeout -k 10 300 python -u bench.py $LEGS --inference-steps 0 > "$O/lab_$v$r.json" 2> "$O/lab_$v$r.err" ;;
    esac || { echo "bench $v failed"; tail -5 "$O/lab_$v$r.err"; exit 1; }
    python3 -c "
import json; d=json.loads(open('$O/lab_$v$r.json').read().strip().splitlines()[-1])
s=d['phase_ms_per_launch_solo']
print('$v', d['value'], d['median_ms_per_step'], 'solo pre/fwd/bwd/gbwd', s['preprocess'], s['render_fwd'], s['render_bwd'], s['gauss_bwd'], 'step bwd', d['phase_ms_per_launch']['render_bwd'])"
  done
done
