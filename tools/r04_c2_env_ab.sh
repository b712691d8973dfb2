#!/bin/bash
# A/B an environment switch on the C2 leg alone (tools/c2_only.py), alternated
# usage: bash tools/r04_c2_env_ab.sh "VAR=value ..." [reps] [steps]
set -u
mkdir -p gpurun_out/r04
E=$1; N=${2:-4}; S=${3:-100}
for r in $(seq $N); do
  echo "def $(timeout -k 10 120 python -u tools/c2_only.py $S 2>/dev/null | grep -v amdgpu | tail -2 | tr "\n" " ")" || exit 1
  echo "$E $(env $E timeout -k 10 120 python -u tools/c2_only.py $S 2>/dev/null | grep -v amdgpu | tail -2 | tr "\n" " ")" || exit 1
done
