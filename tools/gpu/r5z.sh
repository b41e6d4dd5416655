#!/bin/bash
# r5z: k_describe table loads issued after the level-count load (the scan waits for the counts alone)
set -uo pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_golden.py -x -q -m gpu --timeout 200 --timeout-method thread > gpurun_out/r5z_parity.log 2>&1
rc=$?; tail -2 gpurun_out/r5z_parity.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 600 bash tools/ab_bench.sh r5z 3 orb_slam_2_ros_amd/liborbx_head.so orb_slam_2_ros_amd/liborbx.so || exit 1
