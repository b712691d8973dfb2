# A/B of libgsr variants built with `make -C animating-gaussian-splats_amd/csrc variant NAME=x DEFS=...`
# (tools/ab/libgsr_x.so): the default bench step (3 streams) and a one-stream step per variant,
# alternating variants twice so box drift shows.  usage (GPU box): bash tools/ab_variants.sh x y ...
set -o pipefail
mkdir -p gpurun_out/ab
for rep in 1 2; do
  for v in "$@"; do
    for st in 3 1; do
      GSR_LIB=$(pwd)/tools/ab/libgsr_$v.so timeout -k 10 200 python -u bench.py --streams $st --steps 40 ${BENCH_ARGS:-} \
        --call-site-steps 0 --loss-steps 0 --densify-steps 0 --io-timesteps 0 --no-cpu-baseline \
        > gpurun_out/ab/$v.$st.$rep.json 2> gpurun_out/ab/$v.$st.$rep.err || { echo "$v failed"; tail -5 gpurun_out/ab/$v.$st.$rep.err; exit 1; }
      python -c "
import json; d=json.loads([l for l in open('gpurun_out/ab/$v.$st.$rep.json') if l.startswith('{')][0])
p=d['phase_ms_per_launch']
print('$v streams=$st rep=$rep value', d['value'], 'ms/step', d['ms_per_step'], 'bwd', round(p['render_bwd']*1e3), 'items', round(p.get('bwd_items',0)*1e3), 'fwd', round(p['render_fwd']*1e3))"
    done
  done
done
