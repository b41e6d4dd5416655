#!/bin/bash
# Extra SQ counter passes over the VGA bench workload (whole-batch, unpipelined
# launches), one rocprofv3 --pmc run per pass, only counters this box lists.
#   tools/pmc_passes.sh TAG "CTR CTR ..." ["CTR ..."]...
set -uo pipefail
TAG=$1; shift
R=$(pwd)
OUT=$R/gpurun_out/pmc_$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
export ORBX_SPLIT=1 ORBX_PIPELINE=0
timeout -k 10 120 rocprofv3 --list-avail > "$OUT/avail.txt" 2>&1 || true
i=0
for pass in "$@"; do
    i=$((i + 1))
    ok=""
    for c in $pass; do grep -q "\b$c\b" "$OUT/avail.txt" && ok="$ok $c"; done
    echo "pass $i:$ok"
    [ -z "$ok" ] && continue
    timeout -s KILL 200 rocprofv3 --pmc $ok -d "$OUT/p$i" -o pmc -- python "$R/bench.py" --steps 3 --warmup 1 \
        --cpu-seconds 0 --no-extras --no-profile > "$OUT/p$i.log" 2>&1 || { echo "pass $i failed"; tail -3 "$OUT/p$i.log"; exit 1; }
done
cd "$R"
python tools/pmc_table.py $(find "$OUT" -name "*results.db") --kernels k_describe k_fast k_resize_w k_quadtree k_search_init
