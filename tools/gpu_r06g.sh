# r06e (suite + A/B vs the pre-re-walk library) then r06f (the 8x8-quarter backward variant)
set -o pipefail
bash tools/gpu_r06e.sh; rc=$?
[ $rc -le 1 ] || exit $rc
bash tools/gpu_r06f.sh
