# Round 6: k_render_bwd<true> grid 32 vs 256 blocks, 6 alternated pairs.
set -o pipefail
O=gpurun_out/r06exb; mkdir -p $O
bash tools/lib_ab.sh $O 6 exb32 base || exit 1
