#!/bin/bash
# near-threshold exact re-evaluation (tools/ab/libgsr_exact.so) vs default: parity flip rates + time
set -u
mkdir -p gpurun_out/r04
for v in def exact; do
  if [ $v = def ]; then L=animating-gaussian-splats_amd/diff_gaussian_rasterization/libgsr.so; else L=tools/ab/libgsr_exact.so; fi
  rm -f gpurun_out/parity_stats.json
  GSR_LIB=$L timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_headline_parity.py > gpurun_out/r04/exact_par_$v.log 2>&1; echo "$v parity rc=$?"; tail -1 gpurun_out/r04/exact_par_$v.log
  cp gpurun_out/parity_stats.json gpurun_out/r04/parity_stats_$v.json 2>/dev/null
done
python3 - <<'PY'
import json
from collections import defaultdict
PIX = {"n_contrib", "final_T", "color", "depth"}
for v in ("def", "exact"):
    try:
        d = json.load(open(f"gpurun_out/r04/parity_stats_{v}.json"))
    except OSError:
        print(v, "no stats"); continue
    pix, grad = defaultdict(float), defaultdict(float)
    for row in d:
        t, f, frac = row[0], row[1], row[2]
        (pix if f in PIX else grad)[t] = max((pix if f in PIX else grad)[t], frac)
    for t in sorted(set(pix) | set(grad)):
        print(v, t.split("::")[-1], "pix %.2e grad %.2e" % (pix[t], grad[t]))
PY
bash tools/r04_lib_ab.sh exact 2
