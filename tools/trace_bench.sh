#!/bin/bash
# Kernel-trace pass over a short bench run, then per-dispatch durations of the
# last step (tools/kernel_times.py):  tools/trace_bench.sh TAG [bench args]
set -euo pipefail
TAG=$1; shift
R=$(pwd)
OUT=$R/gpurun_out/trace_$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT" -o trace -- python "$R/bench.py" --steps 3 --warmup 1 \
    --cpu-seconds 0 --no-extras --no-profile "$@" > "$OUT/run.log" 2>&1
python "$R/tools/kernel_times.py" "$(find "$OUT" -name 'trace_results.db' | head -n 1)" --last 40 > "$OUT/times.txt"
