#!/bin/bash
# r5o: k_describe occupancy probes (8 / 7 / 6 / 5 waves per SIMD) and a no-table-load timing probe
set -uo pipefail
mkdir -p gpurun_out
timeout -k 10 900 bash tools/ab_bench.sh r5o 2 orb_slam_2_ros_amd/liborbx.so orb_slam_2_ros_amd/liborbx_ov7.so orb_slam_2_ros_amd/liborbx_occ6.so orb_slam_2_ros_amd/liborbx_occ5.so orb_slam_2_ros_amd/liborbx_notab.so || exit 1
