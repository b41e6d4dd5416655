#!/bin/bash
# r7m: full GPU suite, the full bench line and smoke() after the last fast-mode BA changes (round 6 end)
set -uo pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gputest_r06g.log 2>&1 || { tail -5 gpurun_out/gputest_r06g.log; exit 1; }
tail -1 gpurun_out/gputest_r06g.log
timeout -k 10 600 python bench.py > gpurun_out/bench_r06g.log 2>&1 || { tail -5 gpurun_out/bench_r06g.log; exit 1; }
tail -c 300 gpurun_out/bench_r06g.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_r06g.log 2>&1 || { tail -5 gpurun_out/smoke_r06g.log; exit 1; }
tail -3 gpurun_out/smoke_r06g.log
