#!/bin/bash
# A/B of mg_set_tuning switches on the C2 bench, one process per setting:  tools/gpu_tune_ab.sh "" "0=128" ...
mkdir -p gpurun_out && export TMPDIR=/tmp
i=0
for t in "$@"; do
  MOEGAN_TUNE="$t" timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-families --secondary "" \
    > gpurun_out/ab_$i.json 2> gpurun_out/ab_$i.log || { tail -5 gpurun_out/ab_$i.log; exit 1; }
  python3 -c "import json,sys; j=json.loads(open('gpurun_out/ab_$i.json').read().splitlines()[-1]); print('tune=[$t]', j['ms_per_step'], 'ms', j['value'])"
  i=$((i+1))
done
