#!/bin/bash
# Round-3 re-entry: the whole -m gpu suite, then the C2 perf snapshot (rocprof stats + family split).
mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r3_suite.log 2>&1
echo "suite rc=$?"; tail -3 gpurun_out/r3_suite.log
TAG=r3a bash tools/gpu_perf_profile.sh
