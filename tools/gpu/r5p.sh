#!/bin/bash
# r5p: k_describe fp8 pattern table (1 load a lane), o-free moment window (3 MFMAs, 3 table loads), occupancy sweep
set -uo pipefail
mkdir -p gpurun_out
# (parity passed in the first run)
# timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_golden.py "tests/test_gpu_bench_configs.py::test_mono_bench_config_b3072" -x -q -m gpu --timeout 200 --timeout-method thread > gpurun_out/r5p_parity.log 2>&1
# rc=$?; tail -3 gpurun_out/r5p_parity.log; [ $rc -eq 0 ] || { grep -n "Error\|assert\|mismatch" gpurun_out/r5p_parity.log | head -20; exit 1; }
timeout -k 10 900 bash tools/ab_bench.sh r5p 2 orb_slam_2_ros_amd/liborbx_fd.so orb_slam_2_ros_amd/liborbx.so orb_slam_2_ros_amd/liborbx_occ9.so orb_slam_2_ros_amd/liborbx_occ7.so || exit 1
