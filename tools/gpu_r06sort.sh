# Round 6: where a forward wave's time goes at C3 (trace build): the in-render sort, the blend walk, the rest.
set -o pipefail
O=gpurun_out/r06sort; mkdir -p $O
timeout -k 10 300 python -u tools/render_trace.py --config C3 --cams 0,13 > $O/trace_c3.txt 2>&1 && grep "fwd\]" $O/trace_c3.txt | cut -c1-200 && cp gpurun_out/trace_fwd_cam0.npy $O/trace_fwd_c3_cam0.npy && cp gpurun_out/trace_fwd_cam13.npy $O/trace_fwd_c3_cam13.npy
