#!/bin/bash
# Official round measurement: default bench (with CPU baseline), rocprofv3 stats, PMC traffic passes.
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python bench.py 2>&1 | tee gpurun_out/bench_full.log || exit 1
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_full -o run --output-format csv -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/prof_full.log 2>&1 || { echo "rocprof stats failed"; exit 1; }
echo "stats ok"
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_fetch -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/pmc_fetch.log 2>&1 || { echo "pmc fetch failed"; exit 1; }
echo "fetch ok"
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_write -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/pmc_write.log 2>&1 || { echo "pmc write failed"; exit 1; }
echo done
