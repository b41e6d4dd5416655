#!/bin/bash
# Same-box A/B of library builds on one bench extra, optionally at another
# stream count: alternates the libraries ROUNDS times, one line each into
# gpurun_out/ab_TAG.txt (value and per-step stage ms).
#   tools/ab_extra.sh TAG ROUNDS KEY[:STREAMS] lib1.so lib2.so@ENV=V ...
# (lib@K=V runs that library with the environment setting K=V)
set -uo pipefail
TAG=$1; ROUNDS=$2; SPEC=$3; shift 3
KEY=${SPEC%%:*}; N=${SPEC#*:}; [ "$N" = "$SPEC" ] && N=0
mkdir -p gpurun_out
OUT=gpurun_out/ab_$TAG.txt
: > "$OUT"
CODE='
import sys, json
sys.path.insert(0, ".")
import bench
key, n = sys.argv[1], int(sys.argv[2])
if n:
    bench.EXTRAS = [(k, m, w, h, nf, n if k == key else b, u) for k, m, w, h, nf, b, u in bench.EXTRAS]
sys.argv = ["bench.py", "--extra", key, "--steps", "20"]
sys.exit(bench.main())
'
for r in $(seq "$ROUNDS"); do
    for spec in "$@"; do
        lib=${spec%%@*}; envs=""; [ "$lib" != "$spec" ] && envs=${spec#*@}
        line=$(env $envs ORBX_LIB_ALLOW_MISSING=1 ORBX_LIB=$PWD/$lib timeout -k 10 150 python -c "$CODE" "$KEY" "$N" 2>/dev/null | grep "^{" | tail -n 1) || exit 1
        python -c "import json,sys; d=json.loads(sys.argv[2]); print(sys.argv[1], round(d['value']), [round(v, 3) for v in d.get('stage_ms', [])])" "$spec" "$line" >> "$OUT"
    done
done
cat "$OUT"
