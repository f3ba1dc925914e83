#!/bin/bash
# Round-4 measurement pass: new-kernel unit tests, isolated probes, the bf16 step parity tests, the C2 bench line and
# the slowest calls per family (all into gpurun_out/; nothing after a failed GPU step runs).
mkdir -p gpurun_out && export TMPDIR=/tmp
T=${TAG:-r4}
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_d0_gpu.py tests/test_ffn_gpu.py tests/test_gemm_gpu.py > gpurun_out/${T}_unit.log 2>&1 || { tail -30 gpurun_out/${T}_unit.log; exit 1; }
timeout -k 10 120 python tools/ffn_bwd_probe.py > gpurun_out/${T}_probe.txt 2>&1 || exit 1
C=256 timeout -k 10 120 python tools/ffn_bwd_probe.py >> gpurun_out/${T}_probe.txt 2>&1 || exit 1
timeout -k 10 120 python tools/wgrad_wide_probe.py > gpurun_out/${T}_wide.txt 2>&1 || exit 1
timeout -k 10 120 python tools/d0_probe.py > gpurun_out/${T}_d0.txt 2>&1 || exit 1
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_step_bf16_gpu.py tests/test_determinism_gpu.py > gpurun_out/${T}_step.log 2>&1 || { tail -30 gpurun_out/${T}_step.log; exit 1; }
timeout -k 10 200 python bench.py --secondary "" --no-cpu-baseline > gpurun_out/${T}_bench.out 2> gpurun_out/${T}_bench.err || exit 1
timeout -k 10 200 python tools/top_calls.py gemm conv_fwd expert_gemm conv_wgrad+fold > gpurun_out/${T}_top.txt 2>&1 || exit 1
tail -3 gpurun_out/${T}_unit.log; cat gpurun_out/${T}_probe.txt gpurun_out/${T}_wide.txt gpurun_out/${T}_d0.txt; tail -2 gpurun_out/${T}_step.log
cut -c1-300 gpurun_out/${T}_bench.out
