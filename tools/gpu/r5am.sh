#!/bin/bash
# r5am: the bench-config tests with the round-5 settings (level pipeline on the large extras, matcher overlap on the mono steps)
set -uo pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_bench_configs.py -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/r5am_test.log 2>&1
rc=$?; tail -2 gpurun_out/r5am_test.log; [ $rc -eq 0 ] || { grep -n "Error\|assert" gpurun_out/r5am_test.log | head; exit 1; }
