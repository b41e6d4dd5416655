#!/bin/bash
# Same-box A/B of runtime switches: alternates bench.py runs (VGA headline, no
# extras) over the given environment settings (one quoted "K=V K2=V2" string
# each), ROUNDS times, one line each into gpurun_out/ab_TAG.txt.
#   tools/ab_env.sh TAG ROUNDS "ORBX_DESC_PERSIST=0" "ORBX_DESC_PERSIST=1"
set -uo pipefail
TAG=$1; ROUNDS=$2; shift 2
mkdir -p gpurun_out
OUT=gpurun_out/ab_$TAG.txt
: > "$OUT"
for r in $(seq "$ROUNDS"); do
    for envs in "$@"; do
        line=$(env $envs timeout -k 10 150 python bench.py --no-extras --cpu-seconds 0 --steps 40 2>/dev/null | tail -n 1) || exit 1
        python -c "import json,sys; d=json.loads(sys.argv[2]); print(sys.argv[1], round(d['value']), {k: round(v, 3) for k, v in d['stage_ms_per_step'].items()})" "$envs" "$line" >> "$OUT"
    done
done
cat "$OUT"
