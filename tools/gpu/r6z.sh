#!/bin/bash
# r6z: fast local BA with the speculative gated build of the next system vs HEAD (same box), BA tests
set -uo pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_ba.py > gpurun_out/r6z_pytest.txt 2>&1 || { tail -40 gpurun_out/r6z_pytest.txt; exit 1; }
tail -3 gpurun_out/r6z_pytest.txt
: > gpurun_out/r6z_ab_ba.txt
for r in 1 2 3; do
  for spec in "liborbx_baold.so|X=0" "liborbx.so|X=0" "liborbx.so|ORBX_BA_SPEC=0"; do
    L=${spec%%|*}; E=${spec#*|}
    echo "$L $E $(env $E ORBX_LIB_ALLOW_MISSING=1 ORBX_LIB=$PWD/orb_slam_2_ros_amd/$L timeout -k 10 120 python tools/ba_fast_probe.py 5 2>/dev/null | tr '\n' ' ')" >> gpurun_out/r6z_ab_ba.txt || exit 1
  done
done
cat gpurun_out/r6z_ab_ba.txt
