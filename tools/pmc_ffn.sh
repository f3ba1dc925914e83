#!/bin/bash
# Two PMC passes over tools/ffn_probe.py (fused expert FFN in isolation); LIB= selects an A/B build.
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-ffn}
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS"
P2="SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_LDS"
i=0
for P in "$P1" "$P2"; do
  i=$((i+1))
  MOEGAN_HIP_LIB=${LIB:-} timeout -k 10 200 rocprofv3 --pmc $P --output-format csv -d gpurun_out/${TAG}_p$i -o run -- python3 tools/ffn_probe.py > gpurun_out/${TAG}_p$i.log 2>&1 || { echo "pass $i failed"; tail -5 gpurun_out/${TAG}_p$i.log; exit 1; }
done
python3 tools/pmc_table.py gpurun_out/${TAG}_p1 gpurun_out/${TAG}_p2
