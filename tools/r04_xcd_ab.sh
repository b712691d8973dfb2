#!/bin/bash
# XCD-grouped chunk slabs (default) vs chunk order (tools/ab/libgsr_xcd0.so): headline, solo phases, WRITE_SIZE
set -u
mkdir -p gpurun_out/r04
LEGS="--call-site-steps 0 --train-steps 0 --loss-steps 0 --densify-steps 0 --io-timesteps 0 --unchanged-steps 0 --c2-steps 0 --no-cpu-baseline"
for r in 1 2; do
  for v in def xcd0; do
    if [ $v = def ]; then L=""; else L="tools/ab/libgsr_xcd0.so"; fi
    GSR_LIB=${L:-animating-gaussian-splats_amd/diff_gaussian_rasterization/libgsr.so} timeout -k 10 300 python -u bench.py $LEGS > gpurun_out/r04/xab_$v$r.json 2>/dev/null || exit 1
    python3 -c "
import json; d=json.loads(open('gpurun_out/r04/xab_$v$r.json').read().strip().splitlines()[-1])
print('$v', d['value'], d['median_ms_per_step'], {k: d['phase_ms_per_launch'][k] for k in ('bin_emit','tile_sort','render_fwd','render_bwd')}, 'solo emit', d['phase_ms_per_launch_solo']['bin_emit'])"
  done
done
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
for v in def xcd0; do
  if [ $v = def ]; then L=$R/animating-gaussian-splats_amd/diff_gaussian_rasterization/libgsr.so; else L=$R/tools/ab/libgsr_xcd0.so; fi
  GSR_LIB=$L timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "bin_emit|tile_sort" --kernel-trace --output-format csv -d $R/gpurun_out/r04/xw_$v -- python3 $R/bench.py $LEGS --steps 20 --warmup 5 > $R/gpurun_out/r04/xw_$v.log 2>&1 || exit 2
done
cd $R
python3 tools/rocprof_summary.py pmc gpurun_out/r04/xw_def gpurun_out/r04/xw_def 2>/dev/null | grep -i "emit\|sort" || true
python3 tools/rocprof_summary.py pmc gpurun_out/r04/xw_xcd0 gpurun_out/r04/xw_xcd0 2>/dev/null | grep -i "emit\|sort" || true
