#!/bin/bash
# Round-3 evidence pass: -m gpu suite + smoke, C2 family profile (rocprof time + PMC traffic), default bench.
mkdir -p gpurun_out && export TMPDIR=/tmp
TAG=${TAG:-r3f}
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 400 --timeout-method thread > gpurun_out/suite_$TAG.log 2>&1
echo "suite rc=$?"; grep -E "^FAILED|passed|failed" gpurun_out/suite_$TAG.log | tail -8
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1
echo "smoke rc=$?"; tail -1 gpurun_out/smoke_$TAG.log
TAG=$TAG bash tools/gpu_families.sh > gpurun_out/fam_$TAG.out 2>&1 || { echo "families failed"; tail -5 gpurun_out/fam_$TAG.out; exit 1; }
echo "families ok"; head -c 300 gpurun_out/fam_bench_$TAG.json; echo
timeout -k 10 900 python3 bench.py > gpurun_out/bench_default_$TAG.json 2> gpurun_out/bench_default_$TAG.log || { tail -5 gpurun_out/bench_default_$TAG.log; exit 1; }
head -c 500 gpurun_out/bench_default_$TAG.json; echo
