#!/bin/bash
# GPU tests, then the hipGraph bench with and without side streams (MOEGAN_SIDE_STREAM A/B).
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?; tail -3 gpurun_out/gpu_tests.log
[ $rc -eq 0 ] || { grep -E "Error|error|assert|FAILED" gpurun_out/gpu_tests.log | head -20; exit 1; }
for side in 1 0; do
  MOEGAN_SIDE_STREAM=$side timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/bench_side$side.json 2> gpurun_out/bench_side$side.log || { tail -20 gpurun_out/bench_side$side.log; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/bench_side$side.json')); print('side=$side', d['value'], 'img/s', d['ms_per_step'], 'ms; roofline', d['roofline']['achieved'], d['roofline']['launches_timed'])"
done
