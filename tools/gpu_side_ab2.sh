#!/bin/bash
# Side-stream A/B on the C2 bench (MOEGAN_SIDE_STREAM), one process per setting, alternating.
mkdir -p gpurun_out && export TMPDIR=/tmp
for i in 0 1 2 3; do
  s=$((i % 2))
  MOEGAN_SIDE_STREAM=$s timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-families --secondary "" \
    > gpurun_out/side_$i.json 2> gpurun_out/side_$i.log || { tail -5 gpurun_out/side_$i.log; exit 1; }
  python3 -c "import json; j=json.loads(open('gpurun_out/side_$i.json').read().splitlines()[-1]); print('side=$s', j['ms_per_step'], 'ms', j['value'])"
done
