#!/bin/bash
# r6j: k_fast's ballots as the compares' own lane masks (no v_cndmask 0/1 + v_cmp
# round trip; liborbx) vs before (liborbx_ballot0): parity, same-box A/B VGA + FHD stereo
set -uo pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r6j_parity.log 2>&1 || { tail -30 gpurun_out/r6j_parity.log; exit 1; }
tail -1 gpurun_out/r6j_parity.log
timeout -k 10 500 bash tools/ab_bench.sh r6j_ballot_vga 3 orb_slam_2_ros_amd/liborbx_ballot0.so orb_slam_2_ros_amd/liborbx.so || exit 1
timeout -k 10 400 bash tools/ab_extra.sh r6j_ballot_fhd_stereo 2 stereo_fhd_1920x1080 orb_slam_2_ros_amd/liborbx_ballot0.so orb_slam_2_ros_amd/liborbx.so || exit 1
