#!/bin/bash
# r6x: FAST cell records carrying the level's pitch and pyramid offset (no dependent level-args load) vs HEAD, same box
set -uo pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_bench_configs.py > gpurun_out/r6x_pytest.txt 2>&1 || { tail -40 gpurun_out/r6x_pytest.txt; exit 1; }
tail -1 gpurun_out/r6x_pytest.txt
timeout -k 10 900 bash tools/ab_bench.sh r6x 3 orb_slam_2_ros_amd/liborbx_cellold.so orb_slam_2_ros_amd/liborbx.so || exit 1
timeout -k 10 600 bash tools/ab_extra.sh r6x_st 2 stereo_fhd_1920x1080 orb_slam_2_ros_amd/liborbx_cellold.so orb_slam_2_ros_amd/liborbx.so || exit 1
