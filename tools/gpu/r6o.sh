#!/bin/bash
# r6o: local BA fast mode -- Cholesky phase clocks and a per-call kernel timeline
set -uo pipefail
R=$PWD; mkdir -p gpurun_out
ORBX_BA_CLOCKS=1 timeout -k 10 120 python tools/ba_fast_probe.py 5 > gpurun_out/r6o_clocks.txt 2>&1 || { tail -5 gpurun_out/r6o_clocks.txt; exit 1; }
cat gpurun_out/r6o_clocks.txt
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/r6o_ba -o ba -- python $R/tools/ba_fast_probe.py 5 > $R/gpurun_out/r6o_ba.log 2>&1 || { tail -5 $R/gpurun_out/r6o_ba.log; exit 1; }
cd $R && python tools/ba_timeline.py $(find gpurun_out/r6o_ba -name "*.db" | head -1) > gpurun_out/r6o_timeline.txt && cat gpurun_out/r6o_timeline.txt
for r in 1 2 3; do
  for L in orb_slam_2_ros_amd/liborbx_baold.so orb_slam_2_ros_amd/liborbx.so; do
    echo "$L $(ORBX_LIB_ALLOW_MISSING=1 ORBX_LIB=$PWD/$L timeout -k 10 120 python tools/ba_fast_probe.py 5 | tr '\n' ' ')" >> gpurun_out/r6o_ab_ba.txt || exit 1
  done
done
cat gpurun_out/r6o_ab_ba.txt
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_ba.py > gpurun_out/r6o_pytest.txt 2>&1 || { tail -30 gpurun_out/r6o_pytest.txt; exit 1; }
tail -1 gpurun_out/r6o_pytest.txt
for r in 1 2; do
  timeout -k 10 300 bash tools/ab_extra.sh r6o_st192_$r 1 stereo_fhd_1920x1080:192 orb_slam_2_ros_amd/liborbx.so || exit 1
  timeout -k 10 300 bash tools/ab_extra.sh r6o_st256_$r 1 stereo_fhd_1920x1080:256 orb_slam_2_ros_amd/liborbx.so || exit 1
done
