#!/bin/bash
# r5ap: batch split 2 / 1 for the EuRoC and KITTI stereo extras after the LDS-free resize (ORBX_SPLIT env)
set -uo pipefail
mkdir -p gpurun_out
L=orb_slam_2_ros_amd/liborbx.so
for K in stereo_euroc_752x480 stereo_kitti_1241x376; do
  timeout -k 10 400 bash tools/ab_extra.sh r5ap_$K 2 $K $L@ORBX_SPLIT=2 $L@ORBX_SPLIT=1 || exit 1
done
