#!/bin/bash
# r6l: the headline's pipeline as bench.py sets it (no environment) against the
# same settings forced by environment, same box; then the k_fast / k_describe
# phase split of the round-6 kernels
set -uo pipefail
mkdir -p gpurun_out
timeout -k 10 600 bash tools/ab_env.sh r6l_pipe_default 2 "ORBX_NONE=0" "ORBX_PIPELINE=1" "ORBX_PIPELINE=2" "ORBX_PIPELINE=2 ORBX_PIPE_EARLY=2 ORBX_PIPE_DESC=1" || exit 1
timeout -k 10 500 bash tools/phase_valu.sh measure r06c > gpurun_out/phase_valu_r06c.txt 2>&1 || { tail -20 gpurun_out/phase_valu_r06c.txt; exit 1; }
tail -16 gpurun_out/phase_valu_r06c.txt
