#!/bin/bash
# Same-box step-level A/B of library tuning slots (MOEGAN_TUNE), two interleaved rounds; prints ms/step per setting.
mkdir -p gpurun_out && export TMPDIR=/tmp
B="python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --secondary= --no-families"
SETS=("" "20=1024" "20=768" "15=1" "16=3" "18=1" "19=4")
for r in 1 2; do
  for i in "${!SETS[@]}"; do
    MOEGAN_TUNE="${SETS[$i]}" timeout -k 10 200 $B > gpurun_out/sw_${r}_$i.json 2>/dev/null || { echo "failed: ${SETS[$i]}"; exit 1; }
  done
done
for i in "${!SETS[@]}"; do
  python3 -c "
import json
v=[json.loads(open(f'gpurun_out/sw_{r}_$i.json').read().strip().splitlines()[-1])['ms_per_step'] for r in (1,2)]
print('tune=[${SETS[$i]}]', v)"
done
