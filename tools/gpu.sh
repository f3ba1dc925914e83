#!/bin/bash
# One parameterised launcher for every GPU-box job (replaces the one-shot tools/gpu_*.sh scripts of rounds 1-4).
#   tools/gpu.sh TAG step [step ...]          e.g. gpurun -- 'tools/gpu.sh r5a suite bench prof'
# Steps (each under its own time limit; the script stops at the first failing step, nothing after it runs):
#   suite        the whole `pytest -m gpu` suite in one process + smoke()          -> gpurun_out/TAG_suite.log
#   tests=F,G    the named test files only (tests/F.py ...)                        -> gpurun_out/TAG_tests.log
#   bench        default C2 bench line (no CPU leg, no secondary configs)          -> gpurun_out/TAG_bench.json
#   c5bench      the C5 bench line (32 experts top-4, MX-fp8 convs)                -> gpurun_out/TAG_c5bench.json
#   fullbench    the driver's default bench (CPU leg + secondary configs)          -> gpurun_out/TAG_fullbench.json
#   prof         rocprofv3 --kernel-trace --stats of a short replayed bench, the family split and the top kernels
#                                                                                  -> gpurun_out/TAG_prof/, TAG_family.*
#   c5prof       the same for the C5 config
#   pmc          PMC traffic passes (FETCH_SIZE, WRITE_SIZE: one counter set per run) -> gpurun_out/TAG_pmc_*
#   issue        SQ issue profile of one eager step (tools/pmc_step_issue.py)      -> gpurun_out/TAG_issue.txt
#   probe=NAME   python tools/NAME.py (isolated kernel probes)                     -> gpurun_out/TAG_NAME.txt
#   tune=SPEC    bench with MOEGAN_TUNE=SPEC (slot=value[,slot=value])             -> gpurun_out/TAG_tune_SPEC.json
#   c5tune=SPEC  the same on the C5 config                                         -> gpurun_out/TAG_c5tune_SPEC.json
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=$1
shift
O=gpurun_out/$TAG
BENCH_ARGS="--no-cpu-baseline --secondary ''"
run() {  # run LIMIT LOG cmd...: one GPU step under its own limit; print the log tail and stop on failure
  local lim=$1 log=$2
  shift 2
  timeout -k 10 "$lim" "$@" > "$log" 2>&1
  local rc=$?
  if [ $rc -ne 0 ]; then
    echo "[gpu.sh] step failed (rc $rc): $*"
    tail -40 "$log"
    exit 1
  fi
}
for step in "$@"; do
  case $step in
    suite)
      run 1100 ${O}_suite.log python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread
      tail -3 ${O}_suite.log
      run 200 ${O}_smoke.log python -c "import __graft_entry__ as g; g.smoke()"
      tail -2 ${O}_smoke.log ;;
    tests=*)
      files=$(echo "${step#tests=}" | tr ',' '\n' | sed 's#^#tests/#; s#$#.py#' | tr '\n' ' ')
      run 900 ${O}_tests.log python -u -m pytest -x -v -s --timeout 300 --timeout-method thread $files
      grep -E "passed|failed|FAILED" ${O}_tests.log | tail -5 ;;
    bench)
      run 300 ${O}_bench.log python bench.py --no-cpu-baseline --secondary ""
      grep '^{' ${O}_bench.log > ${O}_bench.json
      cut -c1-400 ${O}_bench.json ;;
    c5bench)
      run 300 ${O}_c5bench.log python bench.py --config C5 --no-cpu-baseline --secondary ""
      grep '^{' ${O}_c5bench.log > ${O}_c5bench.json
      cut -c1-400 ${O}_c5bench.json ;;
    fullbench)
      run 600 ${O}_fullbench.log python bench.py
      grep '^{' ${O}_fullbench.log > ${O}_fullbench.json
      cut -c1-600 ${O}_fullbench.json ;;
    prof|c5prof)
      extra=""
      fargs=""
      cfgname=C2
      [ "$step" = c5prof ] && extra="--config C5" && fargs="256 32 bf16 fp8" && cfgname=C5
      # with the attribution step (no --no-families): the roofline kernel is chosen, timed and mg_mark-bracketed
      run 400 ${O}_${step}.log rocprofv3 --kernel-trace --stats -d ${O}_${step} -o run --output-format csv -- \
        python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --secondary "" $extra
      grep '^{' ${O}_${step}.log > ${O}_${step}_line.json
      python3 tools/prof_summary.py ${O}_${step}/run_kernel_stats.csv > ${O}_${step}_stats.txt
      FAMILY_LAST=9 python3 tools/family_time.py ${O}_${step}/run_kernel_trace.csv ${O}_${step}_family.json $fargs > ${O}_${step}_family.txt
      python3 tools/roofline_kernel.py $cfgname ${O}_${step}_line.json ${O}_${step}/run_kernel_trace.csv --last 10 > ${O}_${step}_roofk.txt
      cat ${O}_${step}_family.txt
      head -12 ${O}_${step}_roofk.txt ;;
    pmc)
      for c in FETCH_SIZE WRITE_SIZE; do
        run 300 ${O}_pmc_$c.log rocprofv3 --pmc $c -d ${O}_pmc_$c -o run --output-format csv -- \
          python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --secondary "" --eager
      done
      if [ -f ${O}_prof_line.json ]; then  # the roofline kernel's traffic, bracketed by its mg_mark kernels
        python3 tools/roofline_kernel.py C2 ${O}_prof_line.json ${O}_prof/run_kernel_trace.csv --last 10 \
          $(find ${O}_pmc_FETCH_SIZE -name '*counter_collection.csv' | head -1) \
          $(find ${O}_pmc_WRITE_SIZE -name '*counter_collection.csv' | head -1) > ${O}_pmc_roofk.txt
        cat ${O}_pmc_roofk.txt
      fi
      echo "pmc ok" ;;
    issue)  # two SQ passes (at most 8 SQ counters per run) over 3 eager C2 steps
      P1="SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS"
      P2="SQ_WAVE_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES"
      i=1
      for P in "$P1" "$P2"; do
        run 240 ${O}_issue$i.log rocprofv3 --pmc $P -d ${O}_issue$i -o run --output-format csv -- \
          python3 bench.py --eager --steps 2 --warmup 1 --no-cpu-baseline --no-families --secondary ""
        i=$((i + 1))
      done
      f1=$(find ${O}_issue1 -name '*counter_collection.csv' | head -1)
      f2=$(find ${O}_issue2 -name '*counter_collection.csv' | head -1)
      python3 tools/pmc_step_issue.py "$f1" 3 "$f2" > ${O}_issue.txt
      head -30 ${O}_issue.txt ;;
    probe=*)
      name=${step#probe=}
      run 300 ${O}_${name}.txt python3 tools/${name}.py
      cat ${O}_${name}.txt ;;
    tune=*|c5tune=*)
      spec=${step#*tune=}
      cfg=""
      [ "${step%%tune=*}" = c5 ] && cfg="--config C5"
      run 300 ${O}_tune.log env MOEGAN_TUNE="$spec" python bench.py --no-cpu-baseline --secondary "" $cfg
      grep '^{' ${O}_tune.log > "${O}_${step%%=*}_${spec//[,=]/_}.json"
      echo "${step%%=*} $spec: $(cut -c1-200 "${O}_${step%%=*}_${spec//[,=]/_}.json")" ;;
    *)
      echo "[gpu.sh] unknown step $step"; exit 2 ;;
  esac
done
