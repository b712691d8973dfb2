# Round 6: render_fwd walk mask cleared by bit (s_andn2) instead of m & (m - 1) -- alternated A/B, and the
# SALU / VALU counters of both builds.
set -o pipefail
O=gpurun_out/r06n; mkdir -p $O
bash tools/lib_ab.sh $O 4 bitclr def || exit 1
bash tools/pmc_lib.sh $O bitclr sq && bash tools/pmc_lib.sh $O def sq
