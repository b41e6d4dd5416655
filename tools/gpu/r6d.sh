#!/bin/bash
# r6d: k_fast arc score: the min-over-max identity (ORBX_ARC_DIST=1, product),
# the previous four-op blocks (arc4), and packed three-input f16 min/max
# (ORBX_ARC_F16=1, arcf16): parity of each, same-box A/B on VGA + FHD stereo
set -uo pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r6d_parity.log 2>&1 || { tail -30 gpurun_out/r6d_parity.log; exit 1; }
tail -1 gpurun_out/r6d_parity.log
ORBX_LIB=$PWD/orb_slam_2_ros_amd/liborbx_arcf16.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r6d_f16_parity.log 2>&1 || { tail -30 gpurun_out/r6d_f16_parity.log; exit 1; }
tail -1 gpurun_out/r6d_f16_parity.log
timeout -k 10 500 bash tools/ab_bench.sh r6d_arc_vga 2 orb_slam_2_ros_amd/liborbx_arc4.so orb_slam_2_ros_amd/liborbx.so orb_slam_2_ros_amd/liborbx_arcf16.so || exit 1
timeout -k 10 500 bash tools/ab_extra.sh r6d_arc_fhd_stereo 2 stereo_fhd_1920x1080 orb_slam_2_ros_amd/liborbx_arc4.so orb_slam_2_ros_amd/liborbx.so orb_slam_2_ros_amd/liborbx_arcf16.so || exit 1
