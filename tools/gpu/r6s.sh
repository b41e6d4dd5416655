#!/bin/bash
# r6s: local BA uploads through pinned staging vs HEAD (same box), BA tests, phase laps
set -uo pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_ba.py > gpurun_out/r6s_pytest.txt 2>&1 || { tail -40 gpurun_out/r6s_pytest.txt; exit 1; }
tail -1 gpurun_out/r6s_pytest.txt
: > gpurun_out/r6s_ab_ba.txt
for r in 1 2 3; do
  for L in liborbx_baold.so liborbx.so; do
    echo "$L $(ORBX_LIB_ALLOW_MISSING=1 ORBX_LIB=$PWD/orb_slam_2_ros_amd/$L timeout -k 10 120 python tools/ba_fast_probe.py 5 2>/dev/null | tr '\n' ' ')" >> gpurun_out/r6s_ab_ba.txt || exit 1
  done
done
cat gpurun_out/r6s_ab_ba.txt
for L in liborbx_baold.so liborbx.so; do
  ORBX_BA_TIMING=1 ORBX_LIB_ALLOW_MISSING=1 ORBX_LIB=$PWD/orb_slam_2_ros_amd/$L timeout -k 10 120 python tools/ba_fast_probe.py 3 2>&1 | grep "orbx_local_ba ms" | tail -2
done
