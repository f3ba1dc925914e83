#!/bin/bash
# Per-family roofline evidence for the C2 bench step (all into gpurun_out/, copied to profiles/ by hand):
#   1. rocprofv3 --kernel-trace --stats of bench.py (hipGraph replay) -> family_time_$TAG.json (tools/family_time.py)
#   2. two --pmc passes (FETCH_SIZE, WRITE_SIZE) over 3 eager steps -> family_traffic_$TAG.json (tools/family_pmc.py)
#   3. bench.py itself (reads profiles/family_*.json when they match the workload) -> fam_bench_$TAG.json
#   TAG=r2b tools/gpu_families.sh
mkdir -p gpurun_out && export TMPDIR=/tmp
TAG=${TAG:-r2}
B="python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --secondary="
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/fam_prof_$TAG -o run --output-format csv -- $B --no-families > gpurun_out/fam_prof_$TAG.log 2>&1 || { tail -20 gpurun_out/fam_prof_$TAG.log; exit 1; }
FAMILY_LAST=9 python3 tools/family_time.py gpurun_out/fam_prof_$TAG/run_kernel_trace.csv gpurun_out/family_time_$TAG.json
python3 tools/prof_summary.py gpurun_out/fam_prof_$TAG/run_kernel_stats.csv > gpurun_out/stats_$TAG.txt
P="python3 bench.py --eager --steps 2 --warmup 1 --no-cpu-baseline --no-families"
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/fam_fetch_$TAG -o run --output-format csv -- $P > gpurun_out/fam_fetch_$TAG.log 2>&1 || { tail -20 gpurun_out/fam_fetch_$TAG.log; exit 1; }
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/fam_write_$TAG -o run --output-format csv -- $P > gpurun_out/fam_write_$TAG.log 2>&1 || { tail -20 gpurun_out/fam_write_$TAG.log; exit 1; }
f=$(find gpurun_out/fam_fetch_$TAG -name '*counter_collection.csv' | head -1)
w=$(find gpurun_out/fam_write_$TAG -name '*counter_collection.csv' | head -1)
python3 tools/family_pmc.py "$f" "$w" 3 gpurun_out/family_traffic_$TAG.json
mkdir -p /tmp/fprof && cp gpurun_out/family_time_$TAG.json profiles/family_time.json && cp gpurun_out/family_traffic_$TAG.json profiles/family_traffic.json
timeout -k 10 300 $B > gpurun_out/fam_bench_$TAG.json 2> gpurun_out/fam_bench_$TAG.log || { tail -20 gpurun_out/fam_bench_$TAG.log; exit 1; }
cat gpurun_out/fam_bench_$TAG.json
