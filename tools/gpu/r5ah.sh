#!/bin/bash
# r5ah: direct resize, 10 rows a lane (liborbx, 97 VGPRs) vs 5 rows a lane (liborbx_k5, 57 VGPRs) vs LDS windows (head)
set -uo pipefail
mkdir -p gpurun_out
for L in liborbx liborbx_k5; do
ORBX_LIB=$PWD/orb_slam_2_ros_amd/$L.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -k "pyramid or mvimage" -x -q -m gpu --timeout 200 --timeout-method thread > gpurun_out/r5ah_parity_$L.log 2>&1
rc=$?; tail -1 gpurun_out/r5ah_parity_$L.log; [ $rc -eq 0 ] || exit 1
done
timeout -k 10 600 bash tools/ab_bench.sh r5ah 2 orb_slam_2_ros_amd/liborbx_head.so orb_slam_2_ros_amd/liborbx_k5.so orb_slam_2_ros_amd/liborbx.so || exit 1
