#!/bin/bash
# r6n: settings around the deep pipeline, same box: headline split 1 / 2, batch
# 3072 / 4096; FHD stereo at 192 / 256 pairs; C5 (64 FHD RGB-D streams) and its
# 8-stream rank share with pipeline 0 / 2
set -uo pipefail
mkdir -p gpurun_out
OUT=gpurun_out/ab_r6n_headline.txt
: > $OUT
for r in 1 2; do
  for cfg in "3072|ORBX_NONE=0" "3072|ORBX_SPLIT=2" "4096|ORBX_NONE=0"; do
    b=${cfg%%|*}; e=${cfg#*|}
    line=$(env $e timeout -k 10 200 python bench.py --no-extras --cpu-seconds 0 --steps 40 --batch $b 2>/dev/null | tail -n 1) || exit 1
    python -c "import json,sys; d=json.loads(sys.argv[2]); print(sys.argv[1], round(d['value']), d['ms_per_step'])" "B=$b $e" "$line" >> $OUT
  done
done
cat $OUT
L=orb_slam_2_ros_amd/liborbx.so
timeout -k 10 400 bash tools/ab_extra.sh r6n_fhd_stereo_256 2 stereo_fhd_1920x1080:256 "$L" || exit 1
timeout -k 10 400 bash tools/ab_extra.sh r6n_c5 2 c5 "$L@ORBX_PIPELINE=0" "$L@ORBX_PIPELINE=2" || exit 1
timeout -k 10 400 bash tools/ab_extra.sh r6n_c5_rank8 2 c5_rank8 "$L@ORBX_PIPELINE=0" "$L@ORBX_PIPELINE=2" || exit 1
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_bench_configs.py -k "transitions or deep_level" > gpurun_out/r6n_pytest.txt 2>&1 || { tail -30 gpurun_out/r6n_pytest.txt; exit 1; }
tail -3 gpurun_out/r6n_pytest.txt
