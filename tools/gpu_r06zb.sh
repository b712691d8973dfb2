# Round 6: render-half idempotence (blocking and async forwards).
set -o pipefail
O=gpurun_out/r06zb; mkdir -p $O
timeout -k 10 200 python -u tools/render_half_idem.py > $O/idem.log 2>&1; rc=$?
grep -v amdgpu $O/idem.log | tail -12
exit $rc
