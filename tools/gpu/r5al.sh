#!/bin/bash
# r5al: level pipeline on / off for the FHD RGB-D and KITTI extras after the LDS-free resize (ORBX_PIPELINE env)
set -uo pipefail
mkdir -p gpurun_out
L=orb_slam_2_ros_amd/liborbx.so
for K in rgbd_fhd_1920x1080 stereo_kitti_1241x376; do
  timeout -k 10 400 bash tools/ab_extra.sh r5al_$K 2 $K $L@ORBX_PIPELINE=0 $L@ORBX_PIPELINE=1 || exit 1
done
