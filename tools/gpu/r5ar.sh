#!/bin/bash
# r5ar: internal streams (level pipeline, matcher overlap) on dedicated hardware queues (ORBX_QUEUES=dedicated, CU-mask streams) vs HIP's round-robin queue assignment
set -uo pipefail
mkdir -p gpurun_out
timeout -k 10 900 bash tools/ab_env.sh r5ar 3 "ORBX_QUEUES=default" "ORBX_QUEUES=dedicated" || exit 1
