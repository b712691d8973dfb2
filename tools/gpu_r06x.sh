# Round 6: bisect the async-forward gradient mismatch by gsr_bind part (1 forward, 2 render half, 4 views,
# 8 one-call backward), 5 reps each with the render halves held back.
set -o pipefail
O=gpurun_out/r06x; mkdir -p $O
run() { name=$1; shift; env "$@" timeout -k 10 200 python -u tools/spec_half_repro.py --reps 5 --halves 0 > $O/$name.log 2>&1; echo "== $name $(grep -c 'max 0 n 0; colors_precomp: max 0 n 0' $O/$name.log) ok of $(grep -c '^async' $O/$name.log)"; }
run all15 GSR_NATIVE_BIND=15
run none0 GSR_NATIVE_BIND=0
run fwd1 GSR_NATIVE_BIND=1
run half2 GSR_NATIVE_BIND=2
run views4 GSR_NATIVE_BIND=4
run r05 GSR_LIB=tools/ab/libgsr_r05.so
