#!/bin/bash
# r5q: region pyramid (all levels in one launch) at the bench batch vs the per-level resize kernels
set -uo pipefail
mkdir -p gpurun_out
timeout -k 10 600 bash tools/ab_bench.sh r5q 2 orb_slam_2_ros_amd/liborbx.so orb_slam_2_ros_amd/liborbx_rgn.so || exit 1
