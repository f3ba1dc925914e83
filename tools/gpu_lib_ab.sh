#!/bin/bash
# Same-box step A/B of the HEAD library build (moe-gan_cpsc541_amd/ab_head/, MOEGAN_HIP_LIB) against the working
# tree's, with and without the batched split-K slabs; three interleaved rounds.
mkdir -p gpurun_out && export TMPDIR=/tmp
B="python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --secondary= --no-families"
HEADLIB=$PWD/moe-gan_cpsc541_amd/ab_head/libmoegan_hip.so
LIBS=("$HEADLIB" "" "")
TUNES=("" "" "21=1")
for r in 1 2 3; do
  for i in 0 1 2; do
    MOEGAN_HIP_LIB="${LIBS[$i]}" MOEGAN_TUNE="${TUNES[$i]}" timeout -k 10 200 $B > gpurun_out/ab_${r}_$i.json 2>/dev/null || { echo "failed: $i"; exit 1; }
  done
done
for i in 0 1 2; do
  python3 -c "
import json
v=[json.loads(open(f'gpurun_out/ab_{r}_$i.json').read().strip().splitlines()[-1])['ms_per_step'] for r in (1,2,3)]
print(['head','new','new 21=1'][$i], v)"
done
