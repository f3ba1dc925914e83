mkdir -p gpurun_out; export TMPDIR=/tmp
for v in old new old new; do MOEGAN_HIP_LIB=$PWD/moe-gan_cpsc541_amd/moegan_mi/libmoegan_hip_$v.so timeout -k 10 120 python -u tools/dgrad_probe.py 2>&1 | grep -v amdgpu.ids | sed "s/^/$v /" || exit 1; done
