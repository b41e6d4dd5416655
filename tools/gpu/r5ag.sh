#!/bin/bash
# r5ag: direct resize driven by host column tables + packed 8-byte row records (liborbx) vs aligned direct, in-kernel taps (liborbx_al) vs LDS windows (head)
set -uo pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -k "pyramid or mvimage" -x -q -m gpu --timeout 200 --timeout-method thread > gpurun_out/r5ag_parity.log 2>&1
rc=$?; tail -2 gpurun_out/r5ag_parity.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 600 bash tools/ab_bench.sh r5ag 2 orb_slam_2_ros_amd/liborbx_head.so orb_slam_2_ros_amd/liborbx_al.so orb_slam_2_ros_amd/liborbx.so || exit 1
