#!/bin/bash
mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest -q -s --timeout 400 --timeout-method thread tests/test_step_bf16_gpu.py > gpurun_out/r3_floor.log 2>&1
echo "rc=$?"; grep -E "passed|failed" gpurun_out/r3_floor.log | tail -2
grep -E "temperature gradient|gradient error / bf16 floor" gpurun_out/r3_floor.log | grep -v report | cut -c1-220
