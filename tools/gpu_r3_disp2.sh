#!/bin/bash
mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -q --timeout 200 --timeout-method thread tests/test_dispatch_gpu.py tests/test_batch_gpu.py tests/test_ffn_gpu.py tests/test_router_gpu.py > gpurun_out/r3_disp2_tests.log 2>&1
echo "tests rc=$?"; tail -2 gpurun_out/r3_disp2_tests.log
for c in C2 C5 C2; do
  timeout -k 10 300 python3 bench.py --config $c --steps 20 --warmup 5 --no-cpu-baseline --secondary "" --no-families > gpurun_out/r3_disp2_$c.json 2>/dev/null || exit 1
  python3 -c "import json; d=json.load(open('gpurun_out/r3_disp2_$c.json')); print('$c', d['value'], d['ms_per_step'], d['ms_per_step_median'])"
done
