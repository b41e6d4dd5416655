#!/bin/bash
# r5v: VGA headline batch split x level pipeline sweep after the round-5 kernel cuts (env overrides)
set -uo pipefail
mkdir -p gpurun_out
OUT=gpurun_out/ab_r5v.txt; : > $OUT
for r in 1 2; do
  for cfg in "1 1" "2 1" "2 0" "1 0" "3 1" "4 1"; do
    set -- $cfg
    line=$(ORBX_SPLIT=$1 ORBX_PIPELINE=$2 timeout -k 10 150 python bench.py --no-extras --cpu-seconds 0 --steps 40 2>/dev/null | tail -n 1) || exit 1
    python -c "import json,sys; d=json.loads(sys.argv[2]); print('split/pipe', sys.argv[1], round(d['value']), d['ms_per_step'], {k: round(v, 3) for k, v in d['stage_ms_per_step'].items()})" "$1/$2" "$line" >> $OUT
  done
done
cat $OUT
