#!/bin/bash
# bf16 step parity (deterministic mode, extended floor model) + GEMM pipeline A/B (base vs two-register-stage variants)
mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -v -s --timeout 300 --timeout-method thread tests/test_step_bf16_gpu.py > gpurun_out/r3_bf16d.log 2>&1
echo "bf16 rc=$?"; grep -E "passed|failed" gpurun_out/r3_bf16d.log | tail -2
bash tools/gpu_ab.sh base sb2
