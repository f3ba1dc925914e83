#!/bin/bash
# Same-box step-level A/B of library tuning slots (MOEGAN_TUNE), two interleaved rounds; prints ms/step per setting.
mkdir -p gpurun_out && export TMPDIR=/tmp
B="python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --secondary= --no-families"
SETS=("" "10=256" "10=1024" "7=1" "12=1" "9=2" "13=2" "17=1024" "4=8")
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
