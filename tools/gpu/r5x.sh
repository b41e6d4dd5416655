#!/bin/bash
# r5x: k_resize_w window staging without per-load exec masks (overlapping last pass)
set -uo pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_golden.py "tests/test_gpu_bench_configs.py::test_mono_bench_config_b3072" "tests/test_gpu_bench_configs.py::test_mono_extra_bench_configs" -x -q -m gpu --timeout 200 --timeout-method thread > gpurun_out/r5x_parity.log 2>&1
rc=$?; tail -3 gpurun_out/r5x_parity.log; [ $rc -eq 0 ] || { grep -n "Error\|assert\|mismatch" gpurun_out/r5x_parity.log | head -20; exit 1; }
timeout -k 10 600 bash tools/ab_bench.sh r5x 3 orb_slam_2_ros_amd/liborbx_head.so orb_slam_2_ros_amd/liborbx.so || exit 1
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
ORBX_SPLIT=1 ORBX_PIPELINE=0 timeout -k 10 200 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_ANY SQ_WAVE_CYCLES -d $R/gpurun_out/r5x_sq -o pmc -- python $R/bench.py --steps 3 --warmup 1 --cpu-seconds 0 --no-extras --no-profile > $R/gpurun_out/r5x_sq.log 2>&1 || exit 1
cd $R && python tools/pmc_table.py gpurun_out/r5x_sq/pmc_results.db --kernels k_resize_w
