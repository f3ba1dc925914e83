#!/bin/bash
# A/B of library variants on one GPU box: GEMM probe + short hipGraph bench per variant.
#   tools/gpu_ab.sh v0 v1 ...   (moe-gan_cpsc541_amd/moegan_mi/libmoegan_hip_<v>.so)
mkdir -p gpurun_out
export TMPDIR=/tmp
for v in "$@"; do
  export MOEGAN_HIP_LIB=$PWD/moe-gan_cpsc541_amd/moegan_mi/libmoegan_hip_$v.so
  echo "== $v"
  timeout -k 10 200 python -u tools/gemm_probe.py > gpurun_out/ab_probe_$v.log 2>&1 || { tail -5 gpurun_out/ab_probe_$v.log; exit 1; }
  grep -v amdgpu.ids gpurun_out/ab_probe_$v.log
  timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/ab_bench_$v.json 2> gpurun_out/ab_bench_$v.log || { tail -5 gpurun_out/ab_bench_$v.log; exit 1; }
  python -c "import json,sys; d=json.load(open('gpurun_out/ab_bench_$v.json')); print('bench', d['value'], 'img/s', d['ms_per_step'], 'ms; roofline', d['roofline']['achieved'])"
done
