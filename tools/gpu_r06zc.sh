# Round 6: async-forward gradient mismatch (1 view, held back, busy GPU) under allocator / launch variants.
set -o pipefail
O=gpurun_out/r06zc; mkdir -p $O
run() { name=$1; shift; env "$@" timeout -k 10 200 python -u tools/spec_half_repro.py --reps 2 --views 1 --halves 0 --stash > $O/$name.log 2>&1; echo "== $name"; grep -E '^(async|  rep)' $O/$name.log | cut -c1-160; }
run def GSR_X=0
run nocache PYTORCH_NO_HIP_MEMORY_CACHING=1 PYTORCH_NO_CUDA_MEMORY_CACHING=1
run launchblocking HIP_LAUNCH_BLOCKING=1
run ctypes GSR_NATIVE_BIND=0 GSR_PREALLOC=0
