#!/bin/bash
# r6a: round-6 baseline on one box: the new overlap-transition test first, then
# tools/round_measure.sh (GPU suite, VGA / FHD / FHD-stereo profiles, bench)
set -uo pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_bench_configs.py -k transitions -x -v --timeout 240 --timeout-method thread > gpurun_out/r6a_trans.log 2>&1 || { tail -30 gpurun_out/r6a_trans.log; exit 1; }
tail -2 gpurun_out/r6a_trans.log
bash tools/round_measure.sh r06a
