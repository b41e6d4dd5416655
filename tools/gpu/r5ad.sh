#!/bin/bash
# r5ad: pyramid resize with rows loaded straight from global memory (k_resize_d) vs the LDS windows (head)
set -uo pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_golden.py tests/test_gpu_bench_configs.py -x -q -m gpu --timeout 200 --timeout-method thread > gpurun_out/r5ad_parity.log 2>&1
rc=$?; tail -2 gpurun_out/r5ad_parity.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 600 bash tools/ab_bench.sh r5ad 3 orb_slam_2_ros_amd/liborbx_head.so orb_slam_2_ros_amd/liborbx.so || exit 1
