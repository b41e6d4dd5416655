#!/bin/bash
# r5aq: k_resize_d column-group width per level (fewest wasted columns, the default) vs forced 16 / 32 / 64 lanes a row (ORBX_RS_TWG)
set -uo pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "pyramid" -x -q -m gpu --timeout 200 --timeout-method thread > gpurun_out/r5aq_parity.log 2>&1
rc=$?; tail -1 gpurun_out/r5aq_parity.log; [ $rc -eq 0 ] || exit 1
for T in 16 32 64; do
  ORBX_RS_TWG=$T timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "pyramid and waves and not lds" -x -q -m gpu --timeout 200 --timeout-method thread > gpurun_out/r5aq_parity_$T.log 2>&1
  rc=$?; tail -1 gpurun_out/r5aq_parity_$T.log; [ $rc -eq 0 ] || exit 1
done
timeout -k 10 900 bash tools/ab_env.sh r5aq 2 "ORBX_RS_TWG=0" "ORBX_RS_TWG=16" "ORBX_RS_TWG=32" "ORBX_RS_TWG=64" || exit 1
