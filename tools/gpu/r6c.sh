#!/bin/bash
# r6c: serial MALL-sized chunks (ORBX_CHUNKS) vs the default on the VGA
# headline; the drop-in matchers' per-call latency incl. the C++ projection
# timing (min / median over 1000 calls, ORBX_CALL_TIMING phases)
set -uo pipefail
mkdir -p gpurun_out
timeout -k 10 600 bash tools/ab_env.sh r6c_chunks 2 "ORBX_PIPELINE=1" "ORBX_PIPELINE=0" "ORBX_PIPELINE=0 ORBX_CHUNKS=6" "ORBX_PIPELINE=0 ORBX_CHUNKS=12" || exit 1
timeout -k 10 300 python bench.py --extra matchers > gpurun_out/r6c_matchers.log 2>&1 || { tail -20 gpurun_out/r6c_matchers.log; exit 1; }
tail -c 3000 gpurun_out/r6c_matchers.log
