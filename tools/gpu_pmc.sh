#!/bin/bash
# PMC passes on the isolated roofline kernel (FETCH_SIZE and WRITE_SIZE in separate runs)
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 200 python tools/kernel_probe.py d_conv1 2>&1 | tee gpurun_out/probe.log || exit 1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_probe_fetch -o run --output-format csv -- python3 tools/kernel_probe.py d_conv1 > gpurun_out/pmc_probe_fetch.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_probe_write -o run --output-format csv -- python3 tools/kernel_probe.py d_conv1 > gpurun_out/pmc_probe_write.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_probe -o run --output-format csv -- python3 tools/kernel_probe.py d_conv1 > gpurun_out/prof_probe.log 2>&1 || exit 1
echo done
