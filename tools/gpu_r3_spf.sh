#!/bin/bash
# Build the variant first: copy csrc/*.h + mg_gemm.hip to build/spf_src, apply the patch there (patch -p1 after
# stripping the csrc path), compile mg_gemm.hip and link it with build/obj/*.o into libmoegan_hip_spf1.so.
# A/B of the TAG-2 short-K epilogue prefetch (main build vs libmoegan_hip_spf1.so = the patched build of tools/patches/shortk_epilogue_prefetch.diff), same box.
mkdir -p gpurun_out && export TMPDIR=/tmp
M=$PWD/moe-gan_cpsc541_amd/moegan_mi
for v in "" _spf1; do
  MOEGAN_HIP_LIB=$M/libmoegan_hip$v.so timeout -k 10 200 python -u tools/gemm_probe.py --only d_head_ga1,d_r1_m0v0,d_conv0_fwd,expert_gP > gpurun_out/r3_spf_probe$v.log 2>&1 || exit 1
done
paste gpurun_out/r3_spf_probe.log gpurun_out/r3_spf_probe_spf1.log | grep -v amdgpu
for v in "" _spf1 "" _spf1; do
  MOEGAN_HIP_LIB=$M/libmoegan_hip$v.so timeout -k 10 200 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --secondary "" --no-families > gpurun_out/r3_spf$v.json 2>/dev/null || exit 1
  python3 -c "import json; d=json.load(open('gpurun_out/r3_spf$v.json')); print('main$v', d['value'], d['ms_per_step'], d['ms_per_step_median'], d['roofline']['achieved'])"
done
