#!/bin/bash
# r7k: fast local BA active sets built on the device (usable flags + camera x point -> edge map; no host lists) vs HEAD, same box, laps, BA tests, trace
set -uo pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_ba.py > gpurun_out/r7k_pytest.txt 2>&1 || { tail -40 gpurun_out/r7k_pytest.txt; exit 1; }
tail -1 gpurun_out/r7k_pytest.txt
ORBX_BA_TIMING=1 timeout -k 10 120 python tools/ba_fast_probe.py 3 2>&1 | grep -v amdgpu.ids | tail -4
: > gpurun_out/r7k_ab_ba.txt
for r in 1 2 3; do
  for L in liborbx_baold.so liborbx.so; do
    echo "$L $(ORBX_LIB_ALLOW_MISSING=1 ORBX_LIB=$PWD/orb_slam_2_ros_amd/$L timeout -k 10 120 python tools/ba_fast_probe.py 5 2>/dev/null | tr '\n' ' ')" >> gpurun_out/r7k_ab_ba.txt || exit 1
  done
done
cat gpurun_out/r7k_ab_ba.txt
R=$PWD; cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/r7k_ba -o ba -- python $R/tools/ba_fast_probe.py 5 > $R/gpurun_out/r7k_ba.log 2>&1 || { tail -5 $R/gpurun_out/r7k_ba.log; exit 1; }
cd $R && python tools/ba_timeline.py $(find gpurun_out/r7k_ba -name "*.db" | head -1) > gpurun_out/r7k_timeline.txt && head -30 gpurun_out/r7k_timeline.txt
