#!/bin/bash
# r5ab: local BA fast mode with its trial sums reduced on the device (32 bytes back a trial)
set -uo pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_ba.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/r5ab_ba.log 2>&1
rc=$?; tail -3 gpurun_out/r5ab_ba.log; [ $rc -eq 0 ] || { grep -n "Error\|assert" gpurun_out/r5ab_ba.log | head; exit 1; }
timeout -k 10 300 python -c "import bench, json; print(json.dumps(bench.local_ba_latency(5)))" > gpurun_out/r5ab_ba_bench.log 2>&1 || { tail -5 gpurun_out/r5ab_ba_bench.log; exit 1; }
cat gpurun_out/r5ab_ba_bench.log
