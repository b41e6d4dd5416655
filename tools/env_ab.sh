#!/bin/bash
# Same-box A/B of liborbx environment settings on the VGA headline:
#   tools/env_ab.sh TAG ROUNDS "ENV=.. ENV2=.." "ENV=.." ...   ("-" = no extra env)
set -uo pipefail
TAG=$1; ROUNDS=$2; shift 2
mkdir -p gpurun_out
OUT=gpurun_out/env_ab_$TAG.txt
: > "$OUT"
for r in $(seq "$ROUNDS"); do
    for e in "$@"; do
        [ "$e" = "-" ] && e=""
        line=$(env $e timeout -k 10 150 python bench.py --no-extras --cpu-seconds 0 --steps 40 2>/dev/null | tail -n 1) || exit 1
        python -c "import json,sys; d=json.loads(sys.argv[2]); print(repr(sys.argv[1]), round(d['value']))" "$e" "$line" >> "$OUT"
    done
done
cat "$OUT"
