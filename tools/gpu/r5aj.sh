#!/bin/bash
# r5aj: mono-step matcher overlapping the next step's extraction (ORBX_OVERLAP_MATCH=1) vs off
set -uo pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_bench_configs.py -k "overlap or b3072" -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/r5aj_test.log 2>&1
rc=$?; tail -1 gpurun_out/r5aj_test.log; [ $rc -eq 0 ] || { grep -n "Error\|assert" gpurun_out/r5aj_test.log | head; exit 1; }
timeout -k 10 600 bash tools/ab_env.sh r5aj 3 "ORBX_OVERLAP_MATCH=0" "ORBX_OVERLAP_MATCH=1" || exit 1
