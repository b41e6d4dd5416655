#!/bin/bash
# r6g: deep level pipeline (ORBX_PIPELINE=2, E = ORBX_PIPE_EARLY, describe of
# 1..E on the side stream = ORBX_PIPE_DESC) and the describe overlap
# (ORBX_OVERLAP_DESC=1): parity tests, then same-box A/Bs on VGA and FHD stereo
set -uo pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_bench_configs.py -k "deep_level_pipeline or overlap_describe or overlap_transitions" -x -v --timeout 300 --timeout-method thread > gpurun_out/r6g_parity.log 2>&1 || { tail -30 gpurun_out/r6g_parity.log; exit 1; }
tail -3 gpurun_out/r6g_parity.log
timeout -k 10 900 bash tools/ab_env.sh r6g_deep_vga 2 "ORBX_PIPELINE=1" "ORBX_PIPELINE=2 ORBX_PIPE_EARLY=1" "ORBX_PIPELINE=2 ORBX_PIPE_EARLY=2" "ORBX_PIPELINE=2 ORBX_PIPE_EARLY=3" "ORBX_PIPELINE=2 ORBX_PIPE_EARLY=2 ORBX_PIPE_DESC=1" "ORBX_PIPELINE=2 ORBX_PIPE_EARLY=2 ORBX_OVERLAP_DESC=1" "ORBX_PIPELINE=2 ORBX_PIPE_EARLY=2 ORBX_PIPE_DESC=1 ORBX_OVERLAP_DESC=1" || exit 1
L=orb_slam_2_ros_amd/liborbx.so
timeout -k 10 600 bash tools/ab_extra.sh r6g_deep_fhd_stereo 2 stereo_fhd_1920x1080 "$L@ORBX_PIPELINE=1" "$L@ORBX_PIPELINE=2 ORBX_PIPE_EARLY=1" "$L@ORBX_PIPELINE=2 ORBX_PIPE_EARLY=2" "$L@ORBX_PIPELINE=2 ORBX_PIPE_EARLY=3" "$L@ORBX_PIPELINE=2 ORBX_PIPE_EARLY=2 ORBX_PIPE_DESC=1" || exit 1
