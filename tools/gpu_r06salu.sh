# Round 6: the forward's done-threshold update written with the compare's negation
# (one scalar mask op fewer per walked entry) -- alternated A/B against the previous build, SQ counters.
set -o pipefail
O=gpurun_out/r06salu; mkdir -p $O
bash tools/lib_ab.sh $O 3 thrlt prev || exit 1
bash tools/pmc_lib.sh $O thrlt sq && bash tools/pmc_lib.sh $O prev sq
