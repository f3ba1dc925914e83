#!/bin/bash
# One GPU call for a change: the named tests first (verbose), then the whole GPU suite, then the benches.
#   tools/gpu_new.sh "tests/test_a.py tests/test_b.py" "C2 C4"
mkdir -p gpurun_out && export TMPDIR=/tmp
T=${1:-}
CFGS=${2:-C2}
if [ -n "$T" ]; then
  timeout -k 10 600 python -u -m pytest $T -x -v -s --timeout 300 --timeout-method thread > gpurun_out/new_tests.log 2>&1
  rc=$?; tail -25 gpurun_out/new_tests.log
  [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
fi
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?; tail -6 gpurun_out/gpu_tests.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
for c in $CFGS; do
  timeout -k 10 400 python -u bench.py --config $c --steps 10 --warmup 3 --no-cpu-baseline --no-families \
    > gpurun_out/bench_$c.json 2> gpurun_out/bench_$c.log || { tail -20 gpurun_out/bench_$c.log; exit 1; }
  cat gpurun_out/bench_$c.json
done
