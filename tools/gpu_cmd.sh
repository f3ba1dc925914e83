mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" 2>&1 | tail -1 || exit 1
timeout -k 10 500 python bench.py > gpurun_out/bench_full.json 2> gpurun_out/bench_full.log || { tail -5 gpurun_out/bench_full.log; exit 1; }
cat gpurun_out/bench_full.json
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_full -o run --output-format csv -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/prof_full.log 2>&1 || { echo "rocprof stats failed"; exit 1; }
echo stats ok
