#!/bin/bash
# r7t: round-6 final fast local BA kernel trace (per-call span / busy / idle and per-kernel totals) of the committed code
set -uo pipefail
mkdir -p gpurun_out
ORBX_BA_TIMING=1 timeout -k 10 120 python tools/ba_fast_probe.py 3 2>&1 | grep -v amdgpu.ids | tail -4
R=$PWD; cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/r7t_ba -o ba -- python $R/tools/ba_fast_probe.py 5 > $R/gpurun_out/r7t_ba.log 2>&1 || { tail -5 $R/gpurun_out/r7t_ba.log; exit 1; }
cd $R && python tools/ba_timeline.py $(find gpurun_out/r7t_ba -name "*.db" | head -1) > gpurun_out/r7t_timeline.txt && head -40 gpurun_out/r7t_timeline.txt
