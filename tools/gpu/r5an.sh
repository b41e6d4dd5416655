#!/bin/bash
# r5an: VGA headline batch split x level pipeline re-swept with the LDS-free resize and the matcher overlap
set -uo pipefail
mkdir -p gpurun_out
timeout -k 10 900 bash tools/ab_env.sh r5an 2 "ORBX_SPLIT=1 ORBX_PIPELINE=1" "ORBX_SPLIT=2 ORBX_PIPELINE=1" "ORBX_SPLIT=2 ORBX_PIPELINE=0" "ORBX_SPLIT=1 ORBX_PIPELINE=0" "ORBX_SPLIT=2 ORBX_PIPELINE=1 ORBX_STAGGER=1" || exit 1
