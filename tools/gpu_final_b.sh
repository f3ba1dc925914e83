#!/bin/bash
# Round-end check of the final build: the whole GPU suite (one process) + smoke(), then the default bench line.
mkdir -p gpurun_out && export TMPDIR=/tmp
TAG=fin bash tools/gpu_full_suite.sh || exit 1
timeout -k 10 900 python bench.py > gpurun_out/final_bench2.json 2> gpurun_out/final_bench2.err || { tail -20 gpurun_out/final_bench2.err; exit 1; }
head -c 300 gpurun_out/final_bench2.json; echo; grep -o '"secondary".*' gpurun_out/final_bench2.json | head -c 600
