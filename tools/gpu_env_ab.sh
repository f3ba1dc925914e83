#!/bin/bash
# A/B of runtime environment switches on the C2 bench in one call: tools/gpu_env_ab.sh TAG "ENV1" "ENV2" ...
# each ENV a space-separated list of NAME=VALUE pairs ("" = the defaults); one bench line per variant.
mkdir -p gpurun_out
TAG=$1
shift
i=0
for spec in "$@"; do
  log=gpurun_out/${TAG}_env$i.log
  timeout -k 10 300 env $spec python bench.py --no-cpu-baseline --secondary "" > $log 2>&1
  rc=$?
  if [ $rc -ne 0 ]; then echo "[gpu_env_ab] '$spec' failed (rc $rc)"; tail -20 $log; exit 1; fi
  echo "[$spec] $(grep '^{' $log | cut -c1-160)"
  i=$((i + 1))
done
