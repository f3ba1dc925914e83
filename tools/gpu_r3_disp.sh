#!/bin/bash
# Dispatch rewrite + XCD split-K order: parity tests, GEMM probe A/B of the tile order, C2 / C5 bench A/B.
mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -q --timeout 200 --timeout-method thread tests/test_dispatch_gpu.py tests/test_router_gpu.py tests/test_ffn_gpu.py tests/test_batch_gpu.py tests/test_engine_gpu.py > gpurun_out/r3_disp_tests.log 2>&1
echo "tests rc=$?"; tail -3 gpurun_out/r3_disp_tests.log
timeout -k 10 300 python -u tools/gemm_probe.py --only modconv16_wgrad,modconv8_wgrad,d_conv1_wgrad,linear_wgrad_bf16,expert_wgrad,style_wgrad_fp32 --variants "6=0;6=2;6=1" > gpurun_out/r3_xcd_probe.log 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/r3_xcd_probe.log
for t in "" "6=2" "6=1"; do
  MOEGAN_TUNE=$t timeout -k 10 200 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --secondary "" --no-families > gpurun_out/r3_xcd_bench_$t.json 2>/dev/null || exit 1
  python3 -c "import json; d=json.load(open('gpurun_out/r3_xcd_bench_$t.json')); print('tune=$t', d['value'], d['ms_per_step'], d['ms_per_step_median'])"
done
MOEGAN_TUNE="" timeout -k 10 200 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --secondary "" --no-families > gpurun_out/r3_xcd_bench_again.json 2>/dev/null || exit 1
python3 -c "import json; d=json.load(open('gpurun_out/r3_xcd_bench_again.json')); print('tune= (again)', d['value'], d['ms_per_step'], d['ms_per_step_median'])"
timeout -k 10 300 python3 bench.py --config C5 --steps 10 --warmup 3 --no-cpu-baseline --secondary "" --no-families > gpurun_out/r3_c5_disp.json 2>/dev/null || exit 1
python3 -c "import json; d=json.load(open('gpurun_out/r3_c5_disp.json')); print('C5', d['value'], d['ms_per_step'])"
