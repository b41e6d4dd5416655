#!/bin/bash
set -uo pipefail
mkdir -p gpurun_out
timeout -k 10 120 python -u tools/proj_ab.py 1 20 orb_slam_2_ros_amd/liborbx_t0.so:ORBX_PROJ_TAIL=0 > gpurun_out/r5e.txt 2>&1
cat gpurun_out/r5e.txt | tail -20
