#!/bin/bash
# r5k: the full GPU suite and smoke() on the current tree
set -uo pipefail
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r5k_gputest.log 2>&1
rc=$?; tail -3 gpurun_out/r5k_gputest.log; [ $rc -eq 0 ] || { grep -n "FAILED\|Error" gpurun_out/r5k_gputest.log | head; exit 1; }
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" 2>&1 | tail -2
