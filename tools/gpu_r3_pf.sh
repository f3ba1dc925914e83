#!/bin/bash
# A/B of the epilogue operand prefetch (main build vs libmoegan_hip_pf0.so = -DMG_EPI_PREFETCH=0), same box.
mkdir -p gpurun_out && export TMPDIR=/tmp
M=$PWD/moe-gan_cpsc541_amd/moegan_mi
for v in "" _pf0; do
  MOEGAN_HIP_LIB=$M/libmoegan_hip$v.so timeout -k 10 200 python -u tools/gemm_probe.py --only expert_gP,expert_gP_noaux,expert_gX,d_conv1_fwd,gemm4096_bf16,modconv16_fwd,conv4_fwd,modconv8_wgrad > gpurun_out/r3_pf_probe$v.log 2>&1 || exit 1
done
paste gpurun_out/r3_pf_probe.log gpurun_out/r3_pf_probe_pf0.log | grep -v amdgpu
for v in "" _pf0 "" _pf0; do
  MOEGAN_HIP_LIB=$M/libmoegan_hip$v.so timeout -k 10 200 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --secondary "" --no-families > gpurun_out/r3_pf$v.json 2>/dev/null || exit 1
  python3 -c "import json; d=json.load(open('gpurun_out/r3_pf$v.json')); print('main$v', d['value'], d['ms_per_step'], d['ms_per_step_median'], d['roofline']['achieved'])"
done
