#!/bin/bash
# r5y: k_describe staging row offsets in the lane offset (voff + j * 5 pitch) instead of the scalar offset
set -uo pipefail
mkdir -p gpurun_out
ORBX_LIB=$PWD/orb_slam_2_ros_amd/liborbx_dvoff.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu --timeout 200 --timeout-method thread > gpurun_out/r5y_parity.log 2>&1
rc=$?; tail -2 gpurun_out/r5y_parity.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 600 bash tools/ab_bench.sh r5y 3 orb_slam_2_ros_amd/liborbx_head.so orb_slam_2_ros_amd/liborbx_dvoff.so || exit 1
