#!/bin/bash
# r7p: the whole library built with LLVM's max-ilp / max-memory-clause machine schedulers vs the default, same box (VGA headline, FHD stereo)
set -uo pipefail
mkdir -p gpurun_out
timeout -k 10 900 bash tools/ab_bench.sh r7p 2 orb_slam_2_ros_amd/liborbx.so orb_slam_2_ros_amd/liborbx_ilp.so orb_slam_2_ros_amd/liborbx_memclause.so || exit 1
timeout -k 10 600 bash tools/ab_extra.sh r7p_st 1 stereo_fhd_1920x1080 orb_slam_2_ros_amd/liborbx.so orb_slam_2_ros_amd/liborbx_ilp.so orb_slam_2_ros_amd/liborbx_memclause.so || exit 1
