#!/bin/bash
# tests -> quick bench -> rocprof (each GPU step time-limited; stop at the first failure)
mkdir -p gpurun_out
export TMPDIR=/tmp
B=${B:-256}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/gpu_tests.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 400 python bench.py --steps 5 --warmup 2 --batch $B --no-cpu-baseline 2>&1 | tee gpurun_out/bench_quick.log || exit 1
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --batch $B --no-cpu-baseline > gpurun_out/prof.log 2>&1 || { echo "rocprof failed"; exit 1; }
echo done
