mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gemm_gpu.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -k "wide" > gpurun_out/gpu_tests.log 2>&1; rc=$?; tail -3 gpurun_out/gpu_tests.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 200 python -u tools/gemm_probe.py --only d_conv1_fwd --variants '2=0;2=257;2=258;2=259;2=0;2=259' 2>&1 | grep -v amdgpu.ids || exit 1
