#!/bin/bash
# Stride-1 wgrad column loader: kernel tests, probe A/B (MG_TUNE_S1_OFF), bench A/B.
mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -q --timeout 200 --timeout-method thread tests/test_gemm_gpu.py > gpurun_out/r3_s1_tests.log 2>&1
echo "tests rc=$?"; tail -3 gpurun_out/r3_s1_tests.log
timeout -k 10 300 python -u tools/gemm_probe.py --only modconv16_wgrad,modconv8_wgrad,d_conv1_wgrad --variants "12=0;12=1" > gpurun_out/r3_s1_probe.log 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/r3_s1_probe.log
for t in "" "12=1" "" "12=1"; do
  MOEGAN_TUNE=$t timeout -k 10 200 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --secondary "" --no-families > gpurun_out/r3_s1_bench.json 2>/dev/null || exit 1
  python3 -c "import json; d=json.load(open('gpurun_out/r3_s1_bench.json')); print('tune=$t', d['value'], d['ms_per_step'], d['ms_per_step_median'])"
done
