#!/bin/bash
# r5ak: level pipeline on / off for the FHD / HD mono, FHD stereo and EuRoC extras after the LDS-free resize (ORBX_PIPELINE env)
set -uo pipefail
mkdir -p gpurun_out
L=orb_slam_2_ros_amd/liborbx.so
for K in fhd_1920x1080 hd_1280x720 stereo_fhd_1920x1080 stereo_euroc_752x480; do
  timeout -k 10 400 bash tools/ab_extra.sh r5ak_$K 2 $K $L@ORBX_PIPELINE=0 $L@ORBX_PIPELINE=1 || exit 1
done
