#!/bin/bash
# r5d: per-call matcher output paths, one process per library and turn, alternating:
# SearchByProjection ORBX_PROJ_TAIL 1 (HostTail) / 2 (copy + polled query); SearchByBoW ORBX_BOW_TAIL 1 / 2
set -uo pipefail
mkdir -p gpurun_out
L=orb_slam_2_ros_amd
: > gpurun_out/r5d_call_ab.txt
for r in 1 2 3; do
  for spec in $L/liborbx_a.so:ORBX_PROJ_TAIL=1:ORBX_BOW_TAIL=1 $L/liborbx_b.so:ORBX_PROJ_TAIL=2:ORBX_BOW_TAIL=2 $L/liborbx_c.so:ORBX_PROJ_TAIL=0:ORBX_BOW_TAIL=1 $L/liborbx_pre2f4.so; do
    timeout -k 10 120 python -u tools/call_ab.py 1 300 $spec >> gpurun_out/r5d_call_ab.txt 2>&1 || { cat gpurun_out/r5d_call_ab.txt; exit 1; }
  done
done
cat gpurun_out/r5d_call_ab.txt
