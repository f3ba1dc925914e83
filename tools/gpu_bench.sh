#!/bin/bash
# bench + rocprof kernel stats (each GPU step time-limited, stop at first failure)
mkdir -p gpurun_out
export TMPDIR=/tmp
B=${B:-256}
timeout -k 10 400 python bench.py --steps 3 --warmup 2 --batch $B --no-cpu-baseline 2>&1 | tee gpurun_out/bench_quick.log || { echo "quick bench failed"; exit 1; }
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --batch $B --no-cpu-baseline > gpurun_out/prof.log 2>&1 || { echo "rocprof failed rc=$?"; exit 1; }
echo done
