#!/bin/bash
# Narrow (32-channel) conv kernels: unit tests, then the isolated probe (nothing after a failed GPU step runs).
mkdir -p gpurun_out && export TMPDIR=/tmp
T=${TAG:-narrow}
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_narrow_gpu.py > gpurun_out/${T}_unit.log 2>&1 || { tail -40 gpurun_out/${T}_unit.log; exit 1; }
tail -3 gpurun_out/${T}_unit.log
timeout -k 10 180 python tools/narrow_probe.py > gpurun_out/${T}_probe.txt 2>&1 || { cat gpurun_out/${T}_probe.txt; exit 1; }
cat gpurun_out/${T}_probe.txt
