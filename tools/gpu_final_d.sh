#!/bin/bash
# HEAD check: the whole GPU suite + smoke(), then the default bench line.
mkdir -p gpurun_out && export TMPDIR=/tmp
TAG=fin3 bash tools/gpu_full_suite.sh || exit 1
timeout -k 10 900 python bench.py > gpurun_out/final_bench4.json 2> gpurun_out/final_bench4.err || { tail -20 gpurun_out/final_bench4.err; exit 1; }
head -c 300 gpurun_out/final_bench4.json; echo; grep -o '"secondary".*' gpurun_out/final_bench4.json | head -c 500
