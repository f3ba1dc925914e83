#!/bin/bash
# rocprofv3 kernel trace of a short eager bench, summarised per kernel and per (kernel, grid).
#   TAG=r1f tools/gpu_prof.sh
mkdir -p gpurun_out && export TMPDIR=/tmp
TAG=${TAG:-r1}
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG -o run --output-format csv -- python3 bench.py --steps 4 --warmup 2 --no-cpu-baseline --eager > gpurun_out/prof_$TAG.log 2>&1 || { tail -30 gpurun_out/prof_$TAG.log; exit 1; }
f=$(find gpurun_out/prof_$TAG -name '*kernel_trace.csv' | head -1)
s=$(find gpurun_out/prof_$TAG -name '*kernel_stats.csv' | head -1)
cp "$f" gpurun_out/trace_$TAG.csv; cp "$s" gpurun_out/stats_$TAG.csv
python3 tools/trace_summary.py gpurun_out/trace_$TAG.csv 7 70 > gpurun_out/trace_$TAG.txt
head -60 gpurun_out/trace_$TAG.txt
