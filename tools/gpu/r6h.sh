#!/bin/bash
# r6h: GPU suite with the deep pipeline default; then pipeline 0 / 1 / 2 on the
# other extras (same box, alternating)
set -uo pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gputest_r06h.log 2>&1 || { tail -30 gpurun_out/gputest_r06h.log; exit 1; }
tail -2 gpurun_out/gputest_r06h.log
L=orb_slam_2_ros_amd/liborbx.so
for key in fhd_1920x1080 hd_1280x720 rgbd_fhd_1920x1080 stereo_euroc_752x480 stereo_kitti_1241x376; do
    timeout -k 10 400 bash tools/ab_extra.sh r6h_pipe_$key 2 $key "$L@ORBX_PIPELINE=0" "$L@ORBX_PIPELINE=1" "$L@ORBX_PIPELINE=2" || exit 1
done
