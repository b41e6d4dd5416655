#!/bin/bash
# r5aa: k_fast's cell read as five dwords (scalar loads; the 16-bit level field had taken a vector load)
set -uo pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_golden.py -x -q -m gpu --timeout 200 --timeout-method thread > gpurun_out/r5aa_parity.log 2>&1
rc=$?; tail -2 gpurun_out/r5aa_parity.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 600 bash tools/ab_bench.sh r5aa 3 orb_slam_2_ros_amd/liborbx_head.so orb_slam_2_ros_amd/liborbx.so || exit 1
