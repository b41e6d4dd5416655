#!/bin/bash
# r5c: KFDB scan + mono-extra parity; per-call SearchByProjection across revisions
set -uo pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_kfdb.py tests/test_gpu_bench_configs.py -k "kfdb or mono_extra" -x -v -m gpu --timeout 200 --timeout-method thread > gpurun_out/r5c_tests.log 2>&1
rc=$?; tail -4 gpurun_out/r5c_tests.log; [ $rc -eq 0 ] || exit 1
L=orb_slam_2_ros_amd
timeout -k 10 400 python -u tools/proj_ab.py 4 200 $L/liborbx_r3end.so $L/liborbx_pre2f4.so $L/liborbx_post2f4.so $L/liborbx_pre3dc.so $L/liborbx_post3dc.so $L/liborbx_head.so > gpurun_out/r5c_proj_ab.txt 2>&1
rc=$?; cat gpurun_out/r5c_proj_ab.txt; exit $rc
