#!/bin/bash
# One SQ counter pass over 3 eager C2 steps (2 timed + 1 warm-up) -> per-kernel issue profile.
mkdir -p gpurun_out && export TMPDIR=/tmp
TAG=${TAG:-step}
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS"
timeout -s KILL 240 rocprofv3 --pmc $P1 -d gpurun_out/pmcstep_$TAG -o run --output-format csv -- python3 bench.py --eager --steps 2 --warmup 1 --no-cpu-baseline --no-families --secondary "" > gpurun_out/pmcstep_$TAG.log 2>&1 || { tail -20 gpurun_out/pmcstep_$TAG.log; exit 1; }
f=$(find gpurun_out/pmcstep_$TAG -name '*counter_collection.csv' | head -1)
python3 tools/pmc_step_issue.py "$f" 3 > gpurun_out/pmcstep_$TAG.txt
P2="SQ_WAVE_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES"
timeout -s KILL 240 rocprofv3 --pmc $P2 -d gpurun_out/pmcstep2_$TAG -o run --output-format csv -- python3 bench.py --eager --steps 2 --warmup 1 --no-cpu-baseline --no-families --secondary "" > gpurun_out/pmcstep2_$TAG.log 2>&1 || { tail -20 gpurun_out/pmcstep2_$TAG.log; exit 1; }
f2=$(find gpurun_out/pmcstep2_$TAG -name '*counter_collection.csv' | head -1)
python3 tools/pmc_step_issue.py "$f" 3 "$f2" > gpurun_out/pmcstep_$TAG.txt
