#!/bin/bash
# One iteration: new/targeted GPU tests, full GPU suite, hipGraph bench, kernel trace.  Stops at the first failure.
mkdir -p gpurun_out && export TMPDIR=/tmp
TAG=${TAG:-iter}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider ${FIRST:+$FIRST} > gpurun_out/gpu_tests_$TAG.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/gpu_tests_$TAG.log
[ $rc -eq 0 ] || { grep -E "Error|error|assert|FAILED" gpurun_out/gpu_tests_$TAG.log | head -30; exit 1; }
timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.log || { tail -20 gpurun_out/bench_$TAG.log; exit 1; }
cat gpurun_out/bench_$TAG.json
TAG=$TAG bash tools/gpu_prof.sh
