#!/bin/bash
# Dispatch tests + probe, then the C5 family profile and the SQ issue profile (nothing after a failed test step).
mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 200 python -u -m pytest -x -q --timeout 100 --timeout-method thread tests/test_dispatch_gpu.py > gpurun_out/disp.log 2>&1 || { tail -30 gpurun_out/disp.log; exit 1; }
tail -2 gpurun_out/disp.log
timeout -k 10 120 python tools/dispatch_probe.py > gpurun_out/disp_probe.txt 2>&1 || exit 1
grep -v amdgpu gpurun_out/disp_probe.txt
TAG=r4 bash tools/gpu_c5_families.sh > gpurun_out/c5fam_r4.out 2>&1 || { tail -20 gpurun_out/c5fam_r4.out; exit 1; }
tail -c 300 gpurun_out/c5fam_r4.out
TAG=r4 bash tools/gpu_pmc_step.sh > gpurun_out/pmc_r4.out 2>&1 || { tail -20 gpurun_out/pmc_r4.out; exit 1; }
tail -5 gpurun_out/pmcstep_r4.txt
