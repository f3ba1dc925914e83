#!/bin/bash
# One GPU call: parity tests, eager vs hipGraph bench, GEMM probe.  Logs under gpurun_out/.
#   tools/gpu_check.sh [tests|bench|probe|all] ...
# Each GPU step has its own time limit; a step that times out / crashes ends the script.
mkdir -p gpurun_out
export TMPDIR=/tmp
what=${1:-all}
shift || true
run_tests() {
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
    > gpurun_out/gpu_tests.log 2>&1
  local rc=$?
  tail -5 gpurun_out/gpu_tests.log
  return $rc
}
run_bench() {
  timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --eager \
    > gpurun_out/bench_eager.json 2> gpurun_out/bench_eager.log || { tail -20 gpurun_out/bench_eager.log; return 1; }
  cat gpurun_out/bench_eager.json
  timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline \
    > gpurun_out/bench_graph.json 2> gpurun_out/bench_graph.log || { tail -20 gpurun_out/bench_graph.log; return 1; }
  cat gpurun_out/bench_graph.json
  grep -m 3 '^\[bench\]' gpurun_out/bench_graph.log
  return 0
}
run_probe() {
  timeout -k 10 300 python -u tools/gemm_probe.py "$@" > gpurun_out/gemm_probe.log 2>&1 || { tail -20 gpurun_out/gemm_probe.log; return 1; }
  cat gpurun_out/gemm_probe.log
}
case $what in
  tests) run_tests ;;
  bench) run_bench ;;
  probe) run_probe "$@" ;;
  all)
    run_tests
    rc=$?
    # continue past ordinary test failures (1), never past a timeout / crash
    { [ $rc -eq 0 ] || [ $rc -eq 1 ]; } && run_bench && run_probe "$@" ;;
  bp) run_bench && run_probe "$@" ;;
esac
