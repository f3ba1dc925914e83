#!/bin/bash
# PMC counter passes over tools/gemm_probe.py cases (one rocprofv3 pass per counter group).
#   ONLY=modconv16_fwd,d_conv1_fwd TAG=x bash tools/pmc_probe.sh
mkdir -p gpurun_out
export TMPDIR=/tmp
ONLY=${ONLY:-d_conv1_fwd}
TAG=${TAG:-pmc}
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS"
P2="SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_LDS"
i=0
for P in "$P1" "$P2"; do
  i=$((i+1))
  timeout -k 10 200 rocprofv3 --pmc $P --output-format csv -d gpurun_out/${TAG}_p$i -o run -- python3 tools/gemm_probe.py --only $ONLY --iters 3 ${VARIANTS:+--variants "$VARIANTS"} > gpurun_out/${TAG}_p$i.log 2>&1 || { echo "pass $i failed"; tail -5 gpurun_out/${TAG}_p$i.log; exit 1; }
done
python3 tools/pmc_table.py gpurun_out/${TAG}_p1 gpurun_out/${TAG}_p2
