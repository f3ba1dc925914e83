#!/bin/bash
# A/B of the HIP runtime's graph execution modes on the C2 bench (graph replay): packet capture (default: every node
# into one queue) vs parallel graph streams.  Each run under its own time limit; nothing after a failure.
mkdir -p gpurun_out && export TMPDIR=/tmp
B="python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --secondary= --no-families"
timeout -k 10 200 $B > gpurun_out/gq_default.json 2>/dev/null || exit 1
DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 timeout -k 10 200 $B > gpurun_out/gq_nocap.json 2>/dev/null || exit 1
DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 DEBUG_HIP_FORCE_GRAPH_QUEUES=2 timeout -k 10 200 $B > gpurun_out/gq_nocap_q2.json 2>/dev/null || exit 1
DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 DEBUG_HIP_FORCE_GRAPH_QUEUES=4 timeout -k 10 200 $B > gpurun_out/gq_nocap_q4.json 2>/dev/null || exit 1
timeout -k 10 200 python3 bench.py --eager --steps 10 --warmup 3 --no-cpu-baseline --secondary= --no-families > gpurun_out/gq_eager.json 2>/dev/null || exit 1
for f in default nocap nocap_q2 nocap_q4 eager; do python3 -c "import json,sys; d=json.loads(open('gpurun_out/gq_$f.json').read().strip().splitlines()[-1]); print('$f', d['ms_per_step'], d['value'])"; done
