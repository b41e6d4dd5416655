#!/bin/bash
# r5b: k_describe one-region staging -- parity, same-box A/B against HEAD, SQ pass
set -uo pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_golden.py tests/test_gpu_bow.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/r5b_parity.log 2>&1
rc=$?; tail -3 gpurun_out/r5b_parity.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 600 bash tools/ab_bench.sh r5b_descstage 3 orb_slam_2_ros_amd/liborbx_base.so orb_slam_2_ros_amd/liborbx.so || exit 1
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
for L in base new; do
  lib=$R/orb_slam_2_ros_amd/liborbx.so; [ $L = base ] && lib=$R/orb_slam_2_ros_amd/liborbx_base.so
  ORBX_LIB=$lib ORBX_SPLIT=1 ORBX_PIPELINE=0 timeout -k 10 200 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_ANY SQ_WAVE_CYCLES -d $R/gpurun_out/r5b_sq_$L -o pmc -- python $R/bench.py --steps 3 --warmup 1 --cpu-seconds 0 --no-extras --no-profile > $R/gpurun_out/r5b_sq_$L.log 2>&1 || exit 1
done
echo done
