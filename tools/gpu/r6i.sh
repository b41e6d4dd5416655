#!/bin/bash
# r6i: k_describe's sample offsets as unpacked VGPR-operand f32 ops (product)
# vs the packed f32 pairs (descpk): parity, then same-box A/B on VGA and FHD mono
set -uo pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r6i_parity.log 2>&1 || { tail -30 gpurun_out/r6i_parity.log; exit 1; }
tail -1 gpurun_out/r6i_parity.log
timeout -k 10 500 bash tools/ab_bench.sh r6i_desc_vga 3 orb_slam_2_ros_amd/liborbx_descpk.so orb_slam_2_ros_amd/liborbx.so || exit 1
