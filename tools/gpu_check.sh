#!/bin/bash
# GPU validation run: unit + fixture parity tests, smoke, short bench (each step time-limited).
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests -m gpu -x -q -p no:cacheprovider > gpurun_out/gpu_tests.log 2>&1
echo "tests rc=$?" >> gpurun_out/gpu_tests.log
