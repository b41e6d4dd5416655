#!/bin/bash
# Same-box A/B of library builds: alternates bench.py runs (VGA headline,
# no extras) over the given libraries, ROUNDS times, one JSON line each into
# gpurun_out/ab_TAG.txt.   tools/ab_bench.sh TAG ROUNDS lib1.so lib2.so ...
set -uo pipefail
TAG=$1; ROUNDS=$2; shift 2
mkdir -p gpurun_out
OUT=gpurun_out/ab_$TAG.txt
: > "$OUT"
for r in $(seq "$ROUNDS"); do
    for lib in "$@"; do
        line=$(ORBX_LIB_ALLOW_MISSING=1 ORBX_LIB=$PWD/$lib timeout -k 10 150 python bench.py --no-extras --cpu-seconds 0 --steps 40 2>/dev/null | tail -n 1) || exit 1
        python -c "import json,sys; d=json.loads(sys.argv[2]); print(sys.argv[1], round(d['value']), {k: round(v, 3) for k, v in d['stage_ms_per_step'].items()})" "$lib" "$line" >> "$OUT"
    done
done
cat "$OUT"
