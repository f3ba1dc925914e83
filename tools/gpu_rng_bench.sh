#!/bin/bash
# RNG / zero-grad changes: their tests, the step parity tests, then the C2 bench twice.
mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 200 python -u -m pytest -x -q --timeout 100 --timeout-method thread tests/test_rng_gpu.py tests/test_loop_gpu.py > gpurun_out/rng.log 2>&1 || { tail -30 gpurun_out/rng.log; exit 1; }
tail -2 gpurun_out/rng.log
B="python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --secondary= --no-families"
timeout -k 10 200 $B > gpurun_out/rng_b1.json 2>gpurun_out/rng_b1.err || { tail -20 gpurun_out/rng_b1.err; exit 1; }
timeout -k 10 200 $B > gpurun_out/rng_b2.json 2>/dev/null || exit 1
for f in b1 b2; do python3 -c "import json; d=json.loads(open('gpurun_out/rng_$f.json').read().strip().splitlines()[-1]); print('$f', d['ms_per_step'], d['value'], d['finite'])"; done
