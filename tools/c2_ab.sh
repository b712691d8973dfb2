# C2 leg only, current tree vs an exported tree, alternated: bash tools/c2_ab.sh OUTDIR REPS TREE...
set -u
O=$1; N=$2; shift 2; mkdir -p "$O"
LEGS="--steps 1 --warmup 1 --probe-steps 0 --call-site-steps 0 --train-steps 0 --loss-steps 0 --densify-steps 0 --io-timesteps 0 --unchanged-steps 0 --no-cpu-baseline"
EXTRA_DEF="--inference-steps 0"
for r in $(seq "$N"); do
  for v in "$@"; do
    case "$v" in
      def|fast) B="bench.py $EXTRA_DEF" ;;
      lib_*) B="bench.py $EXTRA_DEF" ;;
      *) B=tools/ab/$v/bench.py ;;
    esac
    if [ "$v" = fast ]; then B="bench.py $EXTRA_DEF"; export GSR_EXACT_THRESHOLDS=0; else unset GSR_EXACT_THRESHOLDS; fi
    case "$v" in lib_*) export GSR_LIB=tools/ab/libgsr_${v#lib_}.so ;; *) unset GSR_LIB ;; esac
    timeout -k 10 300 python -u $B $LEGS > "$O/c2_$v$r.json" 2> "$O/c2_$v$r.err" || { echo "bench $v failed"; tail -3 "$O/c2_$v$r.err"; exit 1; }
    python3 -c "
import json; d=json.loads(open('$O/c2_$v$r.json').read().strip().splitlines()[-1]); c=d['c2']
print('$v', c['Msplats_per_s'], c['median_ms_per_step'], c.get('host_ms_per_step_median'))"
  done
done
