#!/bin/bash
# r5l: round-5 measurement: VGA headline profile (trace + FETCH/WRITE/SQ passes, summarised) and the full bench line
set -uo pipefail
TAG=${1:-r05a}
mkdir -p gpurun_out
timeout -k 10 500 bash tools/profile.sh $TAG || exit 1
P=gpurun_out/prof_$TAG
db() { find "$P/$1" -name "*results.db" | head -n 1; }
python tools/prof_summary.py --trace "$(db trace)" --fetch "$(db fetch)" --write "$(db write)" --sq "$(db sq)" \
    --json gpurun_out/traffic_vga_$TAG.json --frames-per-dispatch 3072 --out gpurun_out/prof_$TAG.txt \
    --title "VGA 640x480 B=3072 unsplit ($TAG)" > /dev/null || exit 1
head -12 gpurun_out/prof_$TAG.txt
timeout -k 10 640 python bench.py > gpurun_out/bench_$TAG.log 2>&1 || { tail -5 gpurun_out/bench_$TAG.log; exit 1; }
tail -c 300 gpurun_out/bench_$TAG.log
