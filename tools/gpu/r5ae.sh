#!/bin/bash
# r5ae: direct resize with dword-aligned 12-byte row loads (liborbx_al) vs unaligned 8-byte (liborbx) vs LDS windows (head)
set -uo pipefail
mkdir -p gpurun_out
ORBX_LIB=$PWD/orb_slam_2_ros_amd/liborbx_al.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -k "pyramid or mvimage" -x -q -m gpu --timeout 200 --timeout-method thread > gpurun_out/r5ae_parity.log 2>&1
rc=$?; tail -2 gpurun_out/r5ae_parity.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 600 bash tools/ab_bench.sh r5ae 2 orb_slam_2_ros_amd/liborbx_head.so orb_slam_2_ros_amd/liborbx_al.so orb_slam_2_ros_amd/liborbx.so || exit 1
