#!/bin/bash
# r5u: k_describe moment-table loads hoisted to the kernel start (before the key's scalar chain)
set -uo pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_golden.py "tests/test_gpu_bench_configs.py::test_mono_bench_config_b3072" -x -q -m gpu --timeout 200 --timeout-method thread > gpurun_out/r5u_parity.log 2>&1
rc=$?; tail -3 gpurun_out/r5u_parity.log; [ $rc -eq 0 ] || { grep -n "Error\|assert\|mismatch" gpurun_out/r5u_parity.log | head -20; exit 1; }
timeout -k 10 600 bash tools/ab_bench.sh r5u 3 orb_slam_2_ros_amd/liborbx_head.so orb_slam_2_ros_amd/liborbx.so || exit 1
