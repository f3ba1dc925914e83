#!/bin/bash
# 1x1 conv weight gradients: split count / mode sweep (tuning slots 4 = splits, 7 = atomics mode).
mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 300 python -u tools/gemm_probe.py --only w1x1_16_128,w1x1_16_256,w1x1_8_256,w1x1_4_512,w1x1_16_8,modconv16_wgrad \
  --variants ";4=16;4=32;4=128;4=256;7=1" > gpurun_out/r3_w1.txt 2>&1 || exit 1
grep -v amdgpu gpurun_out/r3_w1.txt
