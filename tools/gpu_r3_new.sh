#!/bin/bash
# New GPU tests of the final round-3 build (grouped GELU' epilogue, drop-in loop) and the loop bench line.
mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread \
  "tests/test_gemm_gpu.py::test_grouped_gelu_grad_epilogue" tests/test_gemm_gpu.py::test_grouped_gemm_and_wgrad \
  tests/test_loop_gpu.py > gpurun_out/r3_newtests.log 2>&1
rc=$?; grep -E "PASSED|FAILED|passed|failed|Error" gpurun_out/r3_newtests.log | tail -20; [ $rc -eq 0 ] || exit 1
timeout -k 10 300 python3 bench.py --config loop --steps 6 --warmup 2 --no-cpu-baseline > gpurun_out/r3_loop.json 2>/dev/null || exit 1
head -c 700 gpurun_out/r3_loop.json
