#!/bin/bash
# Profiles the VGA bench workload on the GPU box: a kernel-trace/stats pass,
# then separate PMC passes (FETCH_SIZE, WRITE_SIZE, SQ counters), as
# MI355X_MICROARCH.md prescribes (no counter pass combined with runtime traces).
#   tools/profile.sh TAG [extra bench.py args]
# Databases land in gpurun_out/prof_TAG/{trace,fetch,write,sq}/.
set -euo pipefail
TAG=$1; shift
R=$(pwd)
OUT=$R/gpurun_out/prof_$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
# whole-batch, unpipelined launches (bench.py otherwise splits the timed batch
# in two and pipelines the levels)
export ORBX_SPLIT=1 ORBX_PIPELINE=0
B=(python "$R/bench.py" --steps 5 --warmup 2 --cpu-seconds 0 --no-extras --no-profile "$@")
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o trace -- "${B[@]}" > "$OUT/trace.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d "$OUT/fetch" -o pmc -- "${B[@]}" > "$OUT/fetch.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d "$OUT/write" -o pmc -- "${B[@]}" > "$OUT/write.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_ANY SQ_WAIT_INST_ANY \
    SQ_WAVE_CYCLES SQ_BUSY_CYCLES -d "$OUT/sq" -o pmc -- "${B[@]}" > "$OUT/sq.log" 2>&1
find "$OUT" -name "*.db" | sort
