#!/bin/bash
# r5ao: k_describe scalar diet (one constant-table block, one sign test for the interior check, 32-bit slot indices) vs head; SQ counters of both
set -uo pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_golden.py -x -q -m gpu --timeout 200 --timeout-method thread > gpurun_out/r5ao_parity.log 2>&1
rc=$?; tail -1 gpurun_out/r5ao_parity.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 600 bash tools/ab_bench.sh r5ao 2 orb_slam_2_ros_amd/liborbx_head.so orb_slam_2_ros_amd/liborbx.so || exit 1
for L in liborbx_head liborbx; do
  ORBX_LIB=$PWD/orb_slam_2_ros_amd/$L.so timeout -k 10 300 bash tools/pmc_passes.sh r5ao_$L "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_WAVE_CYCLES SQ_BUSY_CYCLES" > gpurun_out/r5ao_pmc_$L.txt 2>&1 || exit 1
  echo "== $L"; grep -A9 "^k_describe<false>" gpurun_out/r5ao_pmc_$L.txt
done
