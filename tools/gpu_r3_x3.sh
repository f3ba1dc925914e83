#!/bin/bash
# Split-bf16 fp32 GEMMs: kernel tests, bf16 step parity, determinism, C2 bench A/B (MOEGAN_F32X3=0/1).
mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -q -s --timeout 200 --timeout-method thread tests/test_f32x3_gpu.py > gpurun_out/r3_x3_tests.log 2>&1
echo "x3 tests rc=$?"; grep -E "passed|failed|x3 " gpurun_out/r3_x3_tests.log | tail -30
timeout -k 10 500 python -u -m pytest -q -s --timeout 400 --timeout-method thread tests/test_step_bf16_gpu.py tests/test_determinism_gpu.py tests/test_graph_replay_gpu.py > gpurun_out/r3_x3_step.log 2>&1
echo "step tests rc=$?"; tail -3 gpurun_out/r3_x3_step.log
for v in 0 1 0 1; do
  MOEGAN_F32X3=$v timeout -k 10 200 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --secondary "" --no-families > gpurun_out/r3_x3_bench_$v.json 2>/dev/null || exit 1
  python3 -c "import json; d=json.load(open('gpurun_out/r3_x3_bench_$v.json')); print('x3=$v', d['value'], d['ms_per_step'], d['ms_per_step_median'])"
done
