#!/bin/bash
# Perf snapshot of the C2 step: rocprofv3 kernel trace + stats of a short hipGraph bench, the family split of the
# traced steps (tools/family_time.py), and the slowest event-timed C-ABI calls with their shapes per family.
#   TAG=x tools/gpu_perf_profile.sh
mkdir -p gpurun_out && export TMPDIR=/tmp
TAG=${TAG:-p}
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/pp_$TAG -o run --output-format csv -- \
  python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-families --secondary "" > gpurun_out/pp_$TAG.json 2> gpurun_out/pp_$TAG.log \
  || { tail -20 gpurun_out/pp_$TAG.log; exit 1; }
python3 tools/prof_summary.py gpurun_out/pp_$TAG/run_kernel_stats.csv > gpurun_out/pp_stats_$TAG.txt
python3 tools/family_time.py gpurun_out/pp_$TAG/run_kernel_trace.csv gpurun_out/pp_family_$TAG.json > gpurun_out/pp_family_$TAG.txt
timeout -k 10 200 python3 tools/top_calls.py gemm conv_fwd expert_gemm conv_wgrad+fold elementwise router_aux layernorm bias_colsum im2col_col2im > gpurun_out/pp_top_$TAG.txt 2>&1
head -c 300 gpurun_out/pp_$TAG.json; echo
cat gpurun_out/pp_family_$TAG.txt
