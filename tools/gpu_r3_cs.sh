#!/bin/bash
mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -q --timeout 200 --timeout-method thread tests/test_gemm_gpu.py tests/test_ffn_gpu.py tests/test_modules_gpu.py > gpurun_out/r3_cs_tests.log 2>&1
echo "tests rc=$?"; grep -E "passed|failed|^FAILED|Error" gpurun_out/r3_cs_tests.log | tail -6
timeout -k 10 500 python -u -m pytest -q --timeout 400 --timeout-method thread tests/test_step_bf16_gpu.py tests/test_engine_gpu.py > gpurun_out/r3_cs_step.log 2>&1
echo "step rc=$?"; grep -E "passed|failed|^FAILED" gpurun_out/r3_cs_step.log | tail -6
for c in C2 C2; do
  timeout -k 10 300 python3 bench.py --config $c --steps 20 --warmup 5 --no-cpu-baseline --secondary "" --no-families > gpurun_out/r3_cs_$c.json 2>/dev/null || exit 1
  python3 -c "import json; d=json.load(open('gpurun_out/r3_cs_$c.json')); print('$c', d['value'], d['ms_per_step'], d['ms_per_step_median'])"
done
