# Round 6: async-forward gradient mismatch: the per-Gaussian pass run twice (second after a sync).
set -o pipefail
O=gpurun_out/r06zf; mkdir -p $O
timeout -k 10 200 python -u tools/spec_half_repro.py --reps 2 --views 1 --halves 0 --stash --nofresh --views-twice > $O/twice.log 2>&1; rc=$?
grep -E '^(async|blocking|  rep|  views|Trace|.*Error)' $O/twice.log | cut -c1-260
exit $rc
