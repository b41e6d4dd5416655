#!/bin/bash
# r5s: k_fast occupancy through the survivor-list size: 528 (9 WG/CU), 640 (8), 1024 (7), 1400 (6)
set -uo pipefail
mkdir -p gpurun_out
timeout -k 10 800 bash tools/ab_bench.sh r5s 2 orb_slam_2_ros_amd/liborbx.so orb_slam_2_ros_amd/liborbx_head.so orb_slam_2_ros_amd/liborbx_l1024.so orb_slam_2_ros_amd/liborbx_l1400.so || exit 1
