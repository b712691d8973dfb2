# rocprofv3 kernel trace + stats of one bench config (GPU box), summarised per kernel and per stream.
# usage: bash tools/profile_config.sh <tag> <bench args...>   -> gpurun_out/prof_<tag>/
set -u
tag=$1; shift
R=$(pwd); O=$R/gpurun_out/prof_$tag; mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/trace" -- \
    python3 "$R/bench.py" --no-cpu-baseline --call-site-steps 0 --train-steps 0 --loss-steps 0 --densify-steps 0 --io-timesteps 0 "$@" \
    > "$O/bench.json" 2> "$O/trace.log" || { echo "trace failed rc=$?"; tail -5 "$O/trace.log"; exit 1; }
cd "$R"
python3 tools/rocprof_summary.py trace "$O/trace" --last 20 --out "$O/trace_summary.json" > "$O/trace_summary.txt" && \
python3 tools/stream_paths.py "$O/trace" --frac 0.5 > "$O/stream_paths.txt" && \
cp "$O"/trace/*/*_kernel_stats.csv "$O/kernel_stats.csv" && echo "profile $tag ok"
