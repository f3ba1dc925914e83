#!/bin/bash
# Round-3 GPU batch 2: deterministic mode, the MTM gradient probe, bf16 / replay / progressive parity.
mkdir -p gpurun_out
export TMPDIR=/tmp
T="python -u -m pytest -v -s --timeout 300 --timeout-method thread"
timeout -k 10 300 $T tests/test_determinism_gpu.py > gpurun_out/r3_det.log 2>&1
echo "det rc=$?"
timeout -k 10 200 python -u tools/mtm_grad_probe.py 32 > gpurun_out/mtmg32.log 2>&1
echo "probe rc=$?"
timeout -k 10 500 $T tests/test_step_bf16_gpu.py tests/test_graph_replay_gpu.py tests/test_progressive_gpu.py > gpurun_out/r3_bf16c.log 2>&1
echo "bf16 rc=$?"
