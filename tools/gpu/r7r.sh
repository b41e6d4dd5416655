#!/bin/bash
# r7r: full GPU suite, the full bench line and smoke() at the end of round 6 (after the per-vertex sums tail batching)
set -uo pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gputest_r06i.log 2>&1 || { tail -5 gpurun_out/gputest_r06i.log; exit 1; }
tail -1 gpurun_out/gputest_r06i.log
timeout -k 10 600 python bench.py > gpurun_out/bench_r06i.log 2>&1 || { tail -5 gpurun_out/bench_r06i.log; exit 1; }
tail -c 300 gpurun_out/bench_r06i.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_r06i.log 2>&1 || { tail -5 gpurun_out/smoke_r06i.log; exit 1; }
tail -3 gpurun_out/smoke_r06i.log
