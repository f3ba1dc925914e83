#!/bin/bash
# The whole GPU test suite in one process (as the round-end driver runs it) and smoke(); nothing after a failure.
mkdir -p gpurun_out && export TMPDIR=/tmp
T=${TAG:-full}
timeout -k 10 1000 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/${T}_suite.log 2>&1 || { tail -40 gpurun_out/${T}_suite.log; exit 1; }
tail -3 gpurun_out/${T}_suite.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${T}_smoke.log 2>&1 || { tail -20 gpurun_out/${T}_smoke.log; exit 1; }
tail -3 gpurun_out/${T}_smoke.log
