#!/bin/bash
# r5ac: fast-mode Cholesky on the FP64 matrix cores, panel 16 (liborbx) vs panel 8 (p8)
set -uo pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_ba.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/r5ac_ba.log 2>&1
rc=$?; tail -2 gpurun_out/r5ac_ba.log; [ $rc -eq 0 ] || { grep -n "Error\|assert" gpurun_out/r5ac_ba.log | head; exit 1; }
ORBX_LIB=$PWD/orb_slam_2_ros_amd/liborbx_p8.so timeout -k 10 300 python -u -m pytest tests/test_gpu_ba.py -x -q -m gpu -k fast --timeout 120 --timeout-method thread > gpurun_out/r5ac_ba8.log 2>&1
rc=$?; tail -2 gpurun_out/r5ac_ba8.log; [ $rc -eq 0 ] || exit 1
for L in liborbx liborbx_p8 liborbx_oldchol; do
  ORBX_LIB=$PWD/orb_slam_2_ros_amd/$L.so timeout -k 10 200 python tools/ba_fast_probe.py 5 2>&1 | grep "fast local" | tr '\n' ' '; echo " $L"
done
