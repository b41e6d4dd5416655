#!/bin/bash
# r6b: k_fast 8-even-point pre-test (ORBX_FAST_EVEN8) parity + same-box A/B on
# VGA and FHD stereo; serial MALL-sized chunks (ORBX_CHUNKS) vs the default;
# the forwarders' new KeyFrameDatabase save/load case on the GPU
set -uo pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_forwarders.py -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/r6b_fwd.log 2>&1 || { tail -30 gpurun_out/r6b_fwd.log; exit 1; }
tail -1 gpurun_out/r6b_fwd.log
ORBX_LIB=$PWD/orb_slam_2_ros_amd/liborbx_even8.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r6b_even8_parity.log 2>&1 || { tail -30 gpurun_out/r6b_even8_parity.log; exit 1; }
tail -1 gpurun_out/r6b_even8_parity.log
timeout -k 10 400 bash tools/ab_bench.sh r6b_even8_vga 2 orb_slam_2_ros_amd/liborbx.so orb_slam_2_ros_amd/liborbx_even8.so || exit 1
timeout -k 10 400 bash tools/ab_extra.sh r6b_even8_fhd_stereo 2 stereo_fhd_1920x1080 orb_slam_2_ros_amd/liborbx.so orb_slam_2_ros_amd/liborbx_even8.so || exit 1
timeout -k 10 600 bash tools/ab_env.sh r6b_chunks 2 "ORBX_PIPELINE=1" "ORBX_PIPELINE=0" "ORBX_PIPELINE=0 ORBX_CHUNKS=6" "ORBX_PIPELINE=0 ORBX_CHUNKS=12" || exit 1
