# A/B of the deferred pass with fresh (lazily allocated, overwritten) vs zero-filled gradients: 3 alternated reps of the default step, 250 steps.
set -o pipefail
mkdir -p gpurun_out/abf
for rep in 1 2 3; do
  for fr in 0 1; do
    GSR_FRESH_GRADS=$fr timeout -k 10 200 python -u bench.py --steps 250 --call-site-steps 0 --loss-steps 0 --densify-steps 0 --io-timesteps 0 --no-cpu-baseline > gpurun_out/abf/$fr.$rep.json 2> gpurun_out/abf/$fr.$rep.err || { tail -5 gpurun_out/abf/$fr.$rep.err; exit 1; }
    python -c "import json; d=json.loads([l for l in open('gpurun_out/abf/$fr.$rep.json') if l.startswith('{')][0]); print('fresh $fr', d['value'], d['ms_per_step'], round(d['phase_ms_per_launch_solo']['gauss_bwd']*1e3))"
  done
done
