# Round 6: bisect the async-forward gradient mismatch (held-back render halves wrong every time):
# library / bind / prealloc / thresholds variants of tools/spec_half_repro.py.
set -o pipefail
O=gpurun_out/r06w; mkdir -p $O
run() { name=$1; shift; env "$@" timeout -k 10 200 python -u tools/spec_half_repro.py --reps 2 --halves 0 > $O/$name.log 2>&1; echo "== $name"; grep -v amdgpu $O/$name.log | grep "async" | cut -c1-200; }
run def GSR_X=0
run ctypes GSR_NATIVE_BIND=0
run noprealloc GSR_PREALLOC=0
run fast GSR_EXACT_THRESHOLDS=0
run base GSR_LIB=tools/ab/libgsr_base.so
run nolong GSR_LIB=tools/ab/libgsr_nolong.so
run r05 GSR_LIB=tools/ab/libgsr_r05.so
