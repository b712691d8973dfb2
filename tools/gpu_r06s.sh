# Round 6: per-wave walk counters of the forward (trace build: batches, ticks in the walk, evaluations) on
# C3M view 0, exact and fast thresholds.
set -o pipefail
O=gpurun_out/r06s; mkdir -p $O
timeout -k 10 300 python -u tools/render_trace.py --config C3M --cams 0 > $O/trace_c3m.txt 2>&1 && grep "fwd" $O/trace_c3m.txt | cut -c1-250 && cp gpurun_out/trace_fwd_cam0.npy $O/trace_fwd_exact.npy
GSR_EXACT_THRESHOLDS=0 timeout -k 10 300 python -u tools/render_trace.py --config C3M --cams 0 > $O/trace_c3m_fast.txt 2>&1 && grep "fwd" $O/trace_c3m_fast.txt | cut -c1-250 && cp gpurun_out/trace_fwd_cam0.npy $O/trace_fwd_fast.npy
