set -o pipefail
O=gpurun_out/r06c; mkdir -p $O
timeout -k 10 300 python -u tools/t_drift.py C3 3 > $O/drift_C3.log 2>&1 || exit $?
timeout -k 10 300 python -u tools/t_drift.py C4 3 > $O/drift_C4.log 2>&1 || exit $?
timeout -k 10 300 python -u tools/t_drift.py C2 2 > $O/drift_C2.log 2>&1 || exit $?
grep -v amdgpu.ids $O/drift_*.log
