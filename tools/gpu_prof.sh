mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r1e -o run --output-format csv -- python3 bench.py --steps 4 --warmup 2 --no-cpu-baseline --eager > gpurun_out/prof_r1e.log 2>&1 || { tail -30 gpurun_out/prof_r1e.log; exit 1; }
f=$(find gpurun_out/prof_r1e -name '*kernel_trace.csv' | head -1)
s=$(find gpurun_out/prof_r1e -name '*kernel_stats.csv' | head -1)
cp "$f" gpurun_out/trace_r1e.csv; cp "$s" gpurun_out/stats_r1e.csv
python3 tools/trace_summary.py gpurun_out/trace_r1e.csv 7 70 > gpurun_out/trace_r1e.txt
head -80 gpurun_out/trace_r1e.txt
