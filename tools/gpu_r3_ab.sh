#!/bin/bash
# Same-box A/B of the C2 step: round-2 HEAD (worktree ab_r2/, built in-tree) vs the current tree, and the current
# tree with bf16 prefix GEMMs; then the full -m gpu suite.
mkdir -p gpurun_out && export TMPDIR=/tmp
BQ="--steps 20 --warmup 5 --no-cpu-baseline --secondary '' --no-families"
timeout -k 10 200 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --secondary "" --no-families > gpurun_out/ab_cur1.json 2> gpurun_out/ab_cur1.log || exit 1
(cd ab_r2 && timeout -k 10 200 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --secondary "" --no-families > ../gpurun_out/ab_r2.json 2> ../gpurun_out/ab_r2.log) || exit 1
MOEGAN_PREFIX_BF16=1 timeout -k 10 200 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --secondary "" --no-families > gpurun_out/ab_pbf16.json 2> gpurun_out/ab_pbf16.log || exit 1
timeout -k 10 200 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --secondary "" --no-families > gpurun_out/ab_cur2.json 2> gpurun_out/ab_cur2.log || exit 1
for f in ab_cur1 ab_r2 ab_pbf16 ab_cur2; do python3 -c "import json,sys; d=json.load(open('gpurun_out/$f.json')); print('$f', d['value'], d['ms_per_step'], d['ms_per_step_median'])"; done
timeout -k 10 1000 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/r3_suite2.log 2>&1
echo "suite rc=$?"; tail -5 gpurun_out/r3_suite2.log
