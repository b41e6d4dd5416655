#!/bin/bash
# r6w: fast local BA, back solve by diagonal-block inverses vs HEAD (same box), BA tests, trace, clocks
set -uo pipefail
R=$PWD; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_ba.py > gpurun_out/r6w_pytest.txt 2>&1 || { tail -40 gpurun_out/r6w_pytest.txt; exit 1; }
tail -1 gpurun_out/r6w_pytest.txt
: > gpurun_out/r6w_ab_ba.txt
for r in 1 2 3; do
  for spec in "liborbx_baold.so|X=0" "liborbx.so|X=0" ; do
    L=${spec%%|*}; E=${spec#*|}
    echo "$L $E $(env $E ORBX_LIB_ALLOW_MISSING=1 ORBX_LIB=$PWD/orb_slam_2_ros_amd/$L timeout -k 10 120 python tools/ba_fast_probe.py 5 2>/dev/null | tr '\n' ' ')" >> gpurun_out/r6w_ab_ba.txt || exit 1
  done
done
cat gpurun_out/r6w_ab_ba.txt
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/r6w_ba -o ba -- python $R/tools/ba_fast_probe.py 5 > $R/gpurun_out/r6w_ba.log 2>&1 || { tail -5 $R/gpurun_out/r6w_ba.log; exit 1; }
cd $R && python tools/ba_timeline.py $(find gpurun_out/r6w_ba -name "*.db" | head -1) > gpurun_out/r6w_timeline.txt && head -32 gpurun_out/r6w_timeline.txt
ORBX_BA_CLOCKS=1 timeout -k 10 120 python tools/ba_fast_probe.py 5 2>&1 | grep cycles
