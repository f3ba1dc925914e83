#!/bin/bash
# rocprofv3 kernel trace + stats of a short hipGraph bench (C2 by default); per-kernel summary to gpurun_out/.
#   TAG=x CFG=C2 tools/gpu_quickprof.sh
mkdir -p gpurun_out && export TMPDIR=/tmp
TAG=${TAG:-q}; CFG=${CFG:-C2}
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/qp_$TAG -o run --output-format csv -- \
  python3 bench.py --config $CFG --steps 5 --warmup 2 --no-cpu-baseline --no-families --secondary "" > gpurun_out/qp_$TAG.json 2> gpurun_out/qp_$TAG.log \
  || { tail -20 gpurun_out/qp_$TAG.log; exit 1; }
python3 tools/prof_summary.py gpurun_out/qp_$TAG/run_kernel_stats.csv > gpurun_out/qp_stats_$TAG.txt
cat gpurun_out/qp_$TAG.json | head -c 400; echo
