#!/bin/bash
# Round-3 GPU batch: progressive fp32 probe, the new parity tests, a quick bench A/B of the prefix precision.
mkdir -p gpurun_out
export TMPDIR=/tmp
T="python -u -m pytest -v -s --timeout 300 --timeout-method thread"
timeout -k 10 200 python -u tools/prog_probe.py > gpurun_out/prog_probe.log 2>&1
echo "probe rc=$?"
timeout -k 10 500 $T tests/test_step_bf16_gpu.py tests/test_graph_replay_gpu.py > gpurun_out/r3_bf16.log 2>&1
echo "bf16+replay rc=$?"
timeout -k 10 300 $T tests/test_loop_gpu.py tests/test_prefetch_gpu.py tests/test_step_c4_gpu.py > gpurun_out/r3_loop.log 2>&1
echo "loop rc=$?"
timeout -k 10 200 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --secondary "" --no-families > gpurun_out/r3_bench_prefix32.log 2>&1
echo "bench rc=$?"
MOEGAN_PREFIX_BF16=1 timeout -k 10 200 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --secondary "" --no-families > gpurun_out/r3_bench_prefix16.log 2>&1
echo "bench16 rc=$?"
