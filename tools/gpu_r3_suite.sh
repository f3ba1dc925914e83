#!/bin/bash
# Whole -m gpu suite + smoke, then the C2 perf snapshot.
mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -q --timeout 400 --timeout-method thread > gpurun_out/r3_suite3.log 2>&1
echo "suite rc=$?"; grep -E "^FAILED|passed|failed" gpurun_out/r3_suite3.log | tail -12
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r3_smoke.log 2>&1
echo "smoke rc=$?"; tail -2 gpurun_out/r3_smoke.log
TAG=${TAG:-r3b} bash tools/gpu_perf_profile.sh
