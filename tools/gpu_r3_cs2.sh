#!/bin/bash
mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -q --timeout 200 --timeout-method thread tests/test_gemm_gpu.py -k colsum > gpurun_out/r3_cs2_tests.log 2>&1
echo "tests rc=$?"; tail -1 gpurun_out/r3_cs2_tests.log
for v in 0 1 0 1; do
  MOEGAN_FUSED_COLSUM=$v timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --secondary "" --no-families > gpurun_out/r3_cs2_$v.json 2>/dev/null || exit 1
  python3 -c "import json; d=json.load(open('gpurun_out/r3_cs2_$v.json')); print('fused=$v', d['value'], d['ms_per_step'], d['ms_per_step_median'])"
done
