#!/bin/bash
# r6m: GPU suite + smoke + the full bench line on the current tree
set -uo pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gputest_r06d.log 2>&1 || { tail -30 gpurun_out/gputest_r06d.log; exit 1; }
tail -1 gpurun_out/gputest_r06d.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_r06d.log 2>&1 || { tail -20 gpurun_out/smoke_r06d.log; exit 1; }
tail -2 gpurun_out/smoke_r06d.log
timeout -k 10 600 python bench.py > gpurun_out/bench_r06d.log 2>&1 || { tail -5 gpurun_out/bench_r06d.log; exit 1; }
tail -c 300 gpurun_out/bench_r06d.log
