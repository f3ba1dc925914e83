#!/bin/bash
# C5 (E=32 top-4, MX-fp8 3x3 modulated convs) kernel evidence: rocprofv3 kernel trace + stats of the C5 bench
# (family time incl. conv_fwd_mx8 priced against the 5 PF fp8 peak), FETCH / WRITE PMC passes over eager C5 steps,
# and the same workload with bf16 convs (--experts 32 --topk 4, no fp8) for the A/B.
mkdir -p gpurun_out && export TMPDIR=/tmp
TAG=${TAG:-c5}
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/c5_prof_$TAG -o run --output-format csv -- \
  python3 bench.py --config C5 --steps 10 --warmup 3 --no-cpu-baseline --secondary "" --no-families \
  > gpurun_out/c5_prof_$TAG.log 2>&1 || { tail -20 gpurun_out/c5_prof_$TAG.log; exit 1; }
FAMILY_LAST=9 python3 tools/family_time.py gpurun_out/c5_prof_$TAG/run_kernel_trace.csv gpurun_out/family_time_C5_$TAG.json 256 32 bf16 fp8
python3 tools/prof_summary.py gpurun_out/c5_prof_$TAG/run_kernel_stats.csv > gpurun_out/c5_stats_$TAG.txt
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/c5_fetch_$TAG -o run --output-format csv -- \
  python3 bench.py --config C5 --eager --steps 2 --warmup 1 --no-cpu-baseline --no-families --secondary "" \
  > gpurun_out/c5_fetch_$TAG.log 2>&1 || { tail -20 gpurun_out/c5_fetch_$TAG.log; exit 1; }
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/c5_write_$TAG -o run --output-format csv -- \
  python3 bench.py --config C5 --eager --steps 2 --warmup 1 --no-cpu-baseline --no-families --secondary "" \
  > gpurun_out/c5_write_$TAG.log 2>&1 || { tail -20 gpurun_out/c5_write_$TAG.log; exit 1; }
f=$(find gpurun_out/c5_fetch_$TAG -name '*counter_collection.csv' | head -1)
w=$(find gpurun_out/c5_write_$TAG -name '*counter_collection.csv' | head -1)
python3 tools/family_pmc.py "$f" "$w" 3 gpurun_out/family_traffic_C5_$TAG.json 256 32 bf16 fp8
cp gpurun_out/family_time_C5_$TAG.json profiles/family_time_C5.json
cp gpurun_out/family_traffic_C5_$TAG.json profiles/family_traffic_C5.json
timeout -k 10 300 python3 bench.py --config C5 --steps 10 --warmup 3 --no-cpu-baseline --secondary "" \
  > gpurun_out/c5_bench_$TAG.json 2> gpurun_out/c5_bench_$TAG.log || { tail -20 gpurun_out/c5_bench_$TAG.log; exit 1; }
timeout -k 10 300 python3 bench.py --experts 32 --topk 4 --steps 10 --warmup 3 --no-cpu-baseline --secondary "" \
  --no-families > gpurun_out/c5_bf16_bench_$TAG.json 2> gpurun_out/c5_bf16_bench_$TAG.log || exit 1
head -c 600 gpurun_out/c5_bench_$TAG.json; echo; head -c 400 gpurun_out/c5_bf16_bench_$TAG.json; echo
