#!/bin/bash
# After a kernel change: its unit tests (UNIT, default the narrow convs), the bf16 step parity / determinism tests,
# the C2 bench line and the slowest calls of the conv families (nothing after a failed GPU step runs).
mkdir -p gpurun_out && export TMPDIR=/tmp
T=${TAG:-sb}
UNIT=${UNIT:-tests/test_narrow_gpu.py}
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread $UNIT > gpurun_out/${T}_unit.log 2>&1 || { tail -40 gpurun_out/${T}_unit.log; exit 1; }
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_step_bf16_gpu.py tests/test_determinism_gpu.py > gpurun_out/${T}_step.log 2>&1 || { tail -30 gpurun_out/${T}_step.log; exit 1; }
timeout -k 10 200 python bench.py --secondary "" --no-cpu-baseline > gpurun_out/${T}_bench.out 2> gpurun_out/${T}_bench.err || exit 1
timeout -k 10 200 python tools/top_calls.py ${FAMS:-conv_fwd conv_wgrad+fold gemm} > gpurun_out/${T}_top.txt 2>&1 || exit 1
tail -2 gpurun_out/${T}_unit.log; tail -2 gpurun_out/${T}_step.log
cut -c1-300 gpurun_out/${T}_bench.out
