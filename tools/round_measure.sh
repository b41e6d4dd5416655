#!/bin/bash
# Round-end measurement on the GPU box: full GPU suite, the VGA headline
# profile and the two 1920x1080 profiles (FHD mono, 192 frames; FHD stereo,
# the north-star unit, 192 pairs = 384 frames a launch): trace + PMC passes,
# summarised; then the full bench line.
#   tools/round_measure.sh TAG [--no-tests]
set -uo pipefail
TAG=$1
mkdir -p gpurun_out
if [ "${2:-}" != "--no-tests" ]; then
    timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gputest_$TAG.log 2>&1 || { tail -5 gpurun_out/gputest_$TAG.log; exit 1; }
    tail -1 gpurun_out/gputest_$TAG.log
fi
db() { find "$1/$2" -name "*results.db" | head -n 1; }
summ() {   # summ PROFTAG JSON FRAMES TITLE
    local P=gpurun_out/prof_$1
    python tools/prof_summary.py --trace "$(db $P trace)" --fetch "$(db $P fetch)" --write "$(db $P write)" \
        --sq "$(db $P sq)" --json "$2" --frames-per-dispatch "$3" --out gpurun_out/prof_$1.txt --title "$4" > /dev/null
}
timeout -k 10 400 bash tools/profile.sh $TAG || exit 1
summ $TAG gpurun_out/traffic_vga_$TAG.json 3072 "VGA 640x480 B=3072 unsplit ($TAG)" || exit 1
timeout -k 10 400 bash tools/profile.sh ${TAG}_fhd --extra fhd_1920x1080 || exit 1
summ ${TAG}_fhd gpurun_out/traffic_fhd_$TAG.json 192 "FHD 1920x1080 mono B=192 unsplit ($TAG)" || exit 1
timeout -k 10 400 bash tools/profile.sh ${TAG}_fhd_stereo --extra stereo_fhd_1920x1080 || exit 1
summ ${TAG}_fhd_stereo gpurun_out/traffic_fhd_stereo_$TAG.json 384 \
    "FHD 1920x1080 stereo, 192 pairs = 384 frames a launch, unsplit ($TAG)" || exit 1
timeout -k 10 600 python bench.py > gpurun_out/bench_$TAG.log 2>&1 || { tail -5 gpurun_out/bench_$TAG.log; exit 1; }
tail -c 400 gpurun_out/bench_$TAG.log
