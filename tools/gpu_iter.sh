#!/bin/bash
# One build->measure iteration on the GPU box: parity tests, GEMM probe, quick bench, rocprof kernel stats.
# Each GPU step is time-limited; the script stops at the first failure.
mkdir -p gpurun_out
export TMPDIR=/tmp
B=${B:-256}
TAG=${TAG:-iter}
timeout -k 10 600 python -m pytest tests -m gpu -x -q -p no:cacheprovider > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/gpu_tests.log
[ $rc -eq 0 ] || { grep -E "Error|error|assert|FAILED" gpurun_out/gpu_tests.log | head -20; exit 1; }
timeout -k 10 200 python tools/gemm_probe.py > gpurun_out/probe_$TAG.log 2>&1 || { echo "probe failed"; tail gpurun_out/probe_$TAG.log; exit 1; }
cat gpurun_out/probe_$TAG.log
timeout -k 10 400 python bench.py --steps 10 --warmup 3 --batch $B --no-cpu-baseline > gpurun_out/bench_$TAG.log 2>&1 || { echo "bench failed"; tail gpurun_out/bench_$TAG.log; exit 1; }
tail -1 gpurun_out/bench_$TAG.log
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --batch $B --no-cpu-baseline > gpurun_out/prof_$TAG.log 2>&1 || { echo "rocprof failed"; exit 1; }
echo done
