#!/bin/bash
# r7s: local BA per-vertex sums 16 edges a batch with predication (one round for most points; bit-exact) vs HEAD, same box; BA tests, A/B
set -uo pipefail
mkdir -p gpurun_out
timeout -k 10 120 python -u -m pytest -x -q --timeout 60 --timeout-method thread -m gpu tests/test_gpu_ba.py -k "mono_only_and_empty" > gpurun_out/r7s_first.txt 2>&1 || { tail -30 gpurun_out/r7s_first.txt; exit 1; }
tail -1 gpurun_out/r7s_first.txt
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_ba.py > gpurun_out/r7s_pytest.txt 2>&1 || { tail -30 gpurun_out/r7s_pytest.txt; exit 1; }
tail -1 gpurun_out/r7s_pytest.txt
ORBX_BA_TIMING=1 timeout -k 10 120 python tools/ba_fast_probe.py 3 2>&1 | grep -v amdgpu.ids | tail -4
: > gpurun_out/r7s_ab_ba.txt
for r in 1 2 3; do
  for L in liborbx_baold.so liborbx.so; do
    echo "$L $(ORBX_LIB_ALLOW_MISSING=1 ORBX_LIB=$PWD/orb_slam_2_ros_amd/$L timeout -k 10 120 python tools/ba_fast_probe.py 5 2>/dev/null | tr '\n' ' ')" >> gpurun_out/r7s_ab_ba.txt || exit 1
  done
done
cat gpurun_out/r7s_ab_ba.txt
