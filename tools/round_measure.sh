#!/bin/bash
# Round-end measurement on the GPU box: full GPU suite, the VGA headline
# profile (trace + PMC passes, summarised), then the full bench line.
#   tools/round_measure.sh TAG
set -uo pipefail
TAG=$1
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gputest_$TAG.log 2>&1 || { tail -5 gpurun_out/gputest_$TAG.log; exit 1; }
tail -1 gpurun_out/gputest_$TAG.log
timeout -k 10 400 bash tools/profile.sh $TAG || exit 1
P=gpurun_out/prof_$TAG
db() { find "$P/$1" -name "*results.db" | head -n 1; }
python tools/prof_summary.py --trace "$(db trace)" --fetch "$(db fetch)" --write "$(db write)" --sq "$(db sq)" \
    --json gpurun_out/traffic_vga_$TAG.json --frames-per-dispatch 3072 --out gpurun_out/prof_$TAG.txt \
    --title "VGA 640x480 B=3072 unsplit ($TAG)" > /dev/null || exit 1
timeout -k 10 600 python bench.py > gpurun_out/bench_$TAG.log 2>&1 || { tail -5 gpurun_out/bench_$TAG.log; exit 1; }
tail -c 400 gpurun_out/bench_$TAG.log
