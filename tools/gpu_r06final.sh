# Round 6 final: profiles of the shipped build (kernel trace + stats, HBM PMC, SQ PMC), then the default
# bench line (N=1) and the C3M line.
set -o pipefail
O=gpurun_out/r06final; mkdir -p $O
bash tools/profile_round.sh r06final > $O/profile.log 2>&1 || { cat $O/profile.log; exit 1; }
cat $O/profile.log
head -24 gpurun_out/prof_r06final/trace_summary.txt
cat gpurun_out/prof_r06final/hbm_pmc.txt | head -20
cat gpurun_out/prof_r06final/sq_pmc.txt | head -20
