#!/bin/bash
# GEMM-core setprio on by default: the -m gpu suite + smoke on the main build, then an A/B of s_setprio in the
# fused expert FFN (libmoegan_hip_ffnb.so vs _ffnp.so, same box).
mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r3_suite.log 2>&1
rc=$?; echo "suite rc=$rc"; tail -3 gpurun_out/r3_suite.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r3_smoke.log 2>&1 || exit 1
tail -2 gpurun_out/r3_smoke.log
for v in ffnb ffnp ffnb ffnp; do
  MOEGAN_HIP_LIB=$PWD/moe-gan_cpsc541_amd/moegan_mi/libmoegan_hip_$v.so timeout -k 10 200 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --secondary "" --no-families > gpurun_out/r3_ffnprio_$v.json 2>/dev/null || exit 1
  python3 -c "import json; d=json.load(open('gpurun_out/r3_ffnprio_$v.json')); print('$v', d['value'], d['ms_per_step'], d['ms_per_step_median'], d['roofline']['achieved'])"
done
for v in ffnb ffnp; do
  MOEGAN_HIP_LIB=$PWD/moe-gan_cpsc541_amd/moegan_mi/libmoegan_hip_$v.so timeout -k 10 200 python -u tools/gemm_probe.py --only ffn128_nosave,ffn128_save,gemm4096_bf16,d_conv1_fwd > gpurun_out/r3_${v}_probe.log 2>&1 || exit 1
done
paste gpurun_out/r3_ffnb_probe.log gpurun_out/r3_ffnp_probe.log | grep -v amdgpu
