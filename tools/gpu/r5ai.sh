#!/bin/bash
# r5ai: k_describe row pass with its nine MFMAs issued before the ordered stores (liborbx) vs head; SQ counters of both
set -uo pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_golden.py -x -q -m gpu --timeout 200 --timeout-method thread > gpurun_out/r5ai_parity.log 2>&1
rc=$?; tail -1 gpurun_out/r5ai_parity.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 600 bash tools/ab_bench.sh r5ai 2 orb_slam_2_ros_amd/liborbx_head.so orb_slam_2_ros_amd/liborbx.so || exit 1
for L in liborbx_head liborbx; do
  ORBX_LIB=$PWD/orb_slam_2_ros_amd/$L.so timeout -k 10 300 bash tools/pmc_passes.sh r5ai_$L "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES" > gpurun_out/r5ai_pmc_$L.txt 2>&1 || exit 1
  echo "== $L"; grep -A12 "k_describe<false>\|k_resize_d" gpurun_out/r5ai_pmc_$L.txt | head -30
done
