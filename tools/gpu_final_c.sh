#!/bin/bash
# Final round-4 check after the grouped weight-gradient split change: its probe, the whole GPU suite + smoke(),
# then the default bench line (nothing after a failed step).
mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 200 python tools/gwgrad_probe.py > gpurun_out/gw3.txt 2>&1 || { cat gpurun_out/gw3.txt; exit 1; }
grep -v amdgpu gpurun_out/gw3.txt
TAG=fin2 bash tools/gpu_full_suite.sh || exit 1
timeout -k 10 900 python bench.py > gpurun_out/final_bench3.json 2> gpurun_out/final_bench3.err || { tail -20 gpurun_out/final_bench3.err; exit 1; }
head -c 300 gpurun_out/final_bench3.json; echo; grep -o '"secondary".*' gpurun_out/final_bench3.json | head -c 500
