#!/bin/bash
# Batched-GEMM split-K slabs (tuning slot 21): GEMM parity, the bf16 / fp32 step parity tests, then a same-box
# step-level A/B (automatic / off / 256-block target), three interleaved rounds.
mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 500 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gemm_gpu.py \
  tests/test_step_bf16_gpu.py tests/test_step_edge_gpu.py > gpurun_out/bs_tests.log 2>&1 || { tail -30 gpurun_out/bs_tests.log; exit 1; }
tail -3 gpurun_out/bs_tests.log
B="python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --secondary= --no-families"
SETS=("" "21=1" "21=256")
for r in 1 2 3; do
  for i in "${!SETS[@]}"; do
    MOEGAN_TUNE="${SETS[$i]}" timeout -k 10 200 $B > gpurun_out/bs_${r}_$i.json 2>/dev/null || { echo "failed: ${SETS[$i]}"; exit 1; }
  done
done
for i in "${!SETS[@]}"; do
  python3 -c "
import json
v=[json.loads(open(f'gpurun_out/bs_{r}_$i.json').read().strip().splitlines()[-1])['ms_per_step'] for r in (1,2,3)]
print('tune=[${SETS[$i]}]', v)"
done
