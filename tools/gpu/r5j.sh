#!/bin/bash
# r5j: local BA kernel trace, ordered vs fast mode
set -uo pipefail
R=$PWD; mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/r5j_ba -o ba -- python $R/tools/ba_probe.py 5 > $R/gpurun_out/r5j_ba.log 2>&1 || { tail -5 $R/gpurun_out/r5j_ba.log; exit 1; }
cd $R && tail -1 gpurun_out/r5j_ba.log && python tools/kstats.py $(find gpurun_out/r5j_ba -name "*kernel_stats.csv" | head -1)
