mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1; rc=$?; tail -3 gpurun_out/gpu_tests.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 200 python -u tools/gemm_probe.py --only offset_head16_fwd --variants '2=0;2=64;2=0;2=64' 2>&1 | grep -v amdgpu.ids || exit 1
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline 2>&1 | tail -1
