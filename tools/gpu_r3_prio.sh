#!/bin/bash
mkdir -p gpurun_out && export TMPDIR=/tmp
for v in base prio base prio; do
  MOEGAN_HIP_LIB=$PWD/moe-gan_cpsc541_amd/moegan_mi/libmoegan_hip_$v.so timeout -k 10 200 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --secondary "" --no-families > gpurun_out/r3_prio_$v.json 2>/dev/null || exit 1
  python3 -c "import json; d=json.load(open('gpurun_out/r3_prio_$v.json')); print('$v', d['value'], d['ms_per_step'], d['ms_per_step_median'], d['roofline']['achieved'])"
done
MOEGAN_HIP_LIB=$PWD/moe-gan_cpsc541_amd/moegan_mi/libmoegan_hip_prio.so timeout -k 10 200 python -u tools/gemm_probe.py --only d_conv1_fwd,modconv16_fwd,conv8_fwd,conv4_fwd,modconv8_wgrad,expert_fc1,gemm4096_bf16 > gpurun_out/r3_prio_probe.log 2>&1
MOEGAN_HIP_LIB=$PWD/moe-gan_cpsc541_amd/moegan_mi/libmoegan_hip_base.so timeout -k 10 200 python -u tools/gemm_probe.py --only d_conv1_fwd,modconv16_fwd,conv8_fwd,conv4_fwd,modconv8_wgrad,expert_fc1,gemm4096_bf16 > gpurun_out/r3_base_probe.log 2>&1
paste gpurun_out/r3_base_probe.log gpurun_out/r3_prio_probe.log | grep -v amdgpu
