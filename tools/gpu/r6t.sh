#!/bin/bash
# r6t: full GPU suite and the full bench line after the fast-mode Cholesky
set -uo pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gputest_r06e.log 2>&1 || { tail -5 gpurun_out/gputest_r06e.log; exit 1; }
tail -1 gpurun_out/gputest_r06e.log
timeout -k 10 600 python bench.py > gpurun_out/bench_r06e.log 2>&1 || { tail -5 gpurun_out/bench_r06e.log; exit 1; }
tail -c 300 gpurun_out/bench_r06e.log
