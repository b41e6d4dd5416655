#!/bin/bash
# r5w: the extractor's fork streams on dedicated hardware queues (ORBX_QUEUES=dedicated) vs pooled: headline + stereo extras
set -uo pipefail
mkdir -p gpurun_out
OUT=gpurun_out/ab_r5w.txt; : > $OUT
for r in 1 2; do
  for q in pooled dedicated; do
    line=$(ORBX_QUEUES=$q timeout -k 10 150 python bench.py --no-extras --cpu-seconds 0 --steps 40 2>/dev/null | tail -n 1) || exit 1
    python -c "import json,sys; d=json.loads(sys.argv[2]); print('headline', sys.argv[1], round(d['value']), d['ms_per_step'])" "$q" "$line" >> $OUT || exit 1
    for x in stereo_euroc_752x480 stereo_fhd_1920x1080; do
      line=$(ORBX_QUEUES=$q timeout -k 10 150 python bench.py --extra $x --steps 20 2>/dev/null | tail -n 1) || exit 1
      python -c "import json,sys; d=json.loads(sys.argv[3]); print(sys.argv[2], sys.argv[1], round(d['value']))" "$q" "$x" "$line" >> $OUT || exit 1
    done
  done
done
cat $OUT
