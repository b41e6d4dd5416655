#!/bin/bash
# r6k: ballot A/B (liborbx vs liborbx_ballot0), then the round measurement of
# the current tree (GPU suite, VGA / FHD / FHD-stereo profiles, bench line)
set -uo pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r6j_parity.log 2>&1 || { tail -30 gpurun_out/r6j_parity.log; exit 1; }
tail -1 gpurun_out/r6j_parity.log
timeout -k 10 400 bash tools/ab_bench.sh r6j_ballot_vga 2 orb_slam_2_ros_amd/liborbx_ballot0.so orb_slam_2_ros_amd/liborbx.so || exit 1
timeout -k 10 300 bash tools/ab_extra.sh r6j_ballot_fhd_stereo 2 stereo_fhd_1920x1080 orb_slam_2_ros_amd/liborbx_ballot0.so orb_slam_2_ros_amd/liborbx.so || exit 1
bash tools/round_measure.sh r06b || exit 1
