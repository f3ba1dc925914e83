#!/bin/bash
# Round-3 evidence: C2 families (rocprof time + PMC traffic), C5 families + fp8 A/B, default bench with the CPU
# baseline and secondary lines.
mkdir -p gpurun_out && export TMPDIR=/tmp
TAG=r3 bash tools/gpu_families.sh > gpurun_out/fam_r3.out 2>&1 || { tail -5 gpurun_out/fam_r3.out; exit 1; }
echo "families ok"
TAG=c5r3 bash tools/gpu_c5_families.sh > gpurun_out/c5_r3.out 2>&1 || { tail -5 gpurun_out/c5_r3.out; exit 1; }
echo "c5 ok"; tail -3 gpurun_out/c5_r3.out
timeout -k 10 600 python3 bench.py > gpurun_out/bench_default_r3.json 2> gpurun_out/bench_default_r3.log || { tail -5 gpurun_out/bench_default_r3.log; exit 1; }
head -c 400 gpurun_out/bench_default_r3.json; echo
