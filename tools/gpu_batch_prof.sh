#!/bin/bash
# Kernel stats of the batched GEMMs with and without split-K slabs (tuning slot 21).
mkdir -p gpurun_out && export TMPDIR=/tmp
B="bench.py --steps 5 --warmup 2 --no-cpu-baseline --secondary= --no-families"
MOEGAN_TUNE= timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/bp_on -o run -- python3 $B > gpurun_out/bp_on.log 2>&1 &&
MOEGAN_TUNE=21=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/bp_off -o run -- python3 $B > gpurun_out/bp_off.log 2>&1
