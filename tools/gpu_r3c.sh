#!/bin/bash
# Round-3 batch: bf16 step tests (slope replay, weight-rounded floor), then one SQ issue pass over the step.
mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest -v -s --timeout 500 --timeout-method thread tests/test_step_bf16_gpu.py > gpurun_out/r3c_bf16b.log 2>&1
echo "bf16 tests rc=$?"
TAG=r3c bash tools/gpu_pmc_step.sh && echo "pmc ok"
