#!/bin/bash
# Same-box A/B of the split schedules (ORBX_STAGGER values), VGA headline only.
set -uo pipefail
mkdir -p gpurun_out
OUT=gpurun_out/stagger_ab.txt
: > "$OUT"
for r in 1 2; do
    for sg in "$@"; do
        line=$(ORBX_STAGGER=$sg timeout -k 10 150 python bench.py --no-extras --cpu-seconds 0 --steps 40 2>/dev/null | tail -n 1) || exit 1
        python -c "import json,sys; d=json.loads(sys.argv[2]); print('stagger', sys.argv[1], round(d['value']))" "$sg" "$line" >> "$OUT"
    done
done
cat "$OUT"
