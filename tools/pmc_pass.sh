#!/bin/bash
# One rocprofv3 PMC pass (its own run, no trace domains) over a short bench:
#   tools/pmc_pass.sh TAG "COUNTERS" [bench args]   ->  gpurun_out/pmc_TAG/
set -euo pipefail
TAG=$1; CNT=$2; shift 2
R=$(pwd)
OUT=$R/gpurun_out/pmc_$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
export ORBX_SPLIT=1
timeout -s KILL 120 rocprofv3 --pmc $CNT -d "$OUT" -o pmc -- python "$R/bench.py" --steps 2 --warmup 1 \
    --cpu-seconds 0 --no-extras --no-profile "$@" > "$OUT/run.log" 2>&1
python "$R/tools/pmc_table.py" "$(find "$OUT" -name 'pmc_results.db' | head -n 1)" > "$OUT/table.txt"
