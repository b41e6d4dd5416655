#!/bin/bash
set -uo pipefail
mkdir -p gpurun_out
ORBX_LIB=$PWD/orb_slam_2_ros_amd/liborbx_nod16.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "stages_bit_exact" -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/r5i.log 2>&1
echo "nod16 rc=$?"; tail -2 gpurun_out/r5i.log
