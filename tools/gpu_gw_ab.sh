#!/bin/bash
# Same-box A/B of the grouped weight-gradient split target on the C2 bench: 512 blocks (round-3 rule) vs 256 (default).
mkdir -p gpurun_out && export TMPDIR=/tmp
B="python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --secondary= --no-families"
for i in 1 2; do
  MOEGAN_TUNE=20=512 timeout -k 10 200 $B > gpurun_out/gw_old$i.json 2>/dev/null || exit 1
  timeout -k 10 200 $B > gpurun_out/gw_new$i.json 2>/dev/null || exit 1
done
for f in old1 new1 old2 new2; do python3 -c "import json; d=json.loads(open('gpurun_out/gw_$f.json').read().strip().splitlines()[-1]); print('$f', d['ms_per_step'], d['value'])"; done
