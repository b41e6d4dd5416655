#!/bin/bash
# Pins the VALU issue ceiling and the clock the chip holds under the bench
# (VERDICT r01 item 3): the valu_rate micro-benchmark (s_memtime clock stamps)
# and ONE rocprofv3 PMC pass of GRBM_GUI_ACTIVE / SQ_BUSY_CYCLES / SQ_INSTS_VALU
# / SQ_WAVES / SQ_WAVE_CYCLES over both valu_rate and a short VGA bench, plus a
# kernel-trace pass over the same bench for the durations the counters divide.
#   tools/gpu_clock_pass.sh TAG   ->  gpurun_out/clk_TAG/
set -euo pipefail
TAG=$1
R=$(pwd)
OUT=$R/gpurun_out/clk_$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
export ORBX_SPLIT=1
CNT="GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_WAVES SQ_WAVE_CYCLES"
timeout -k 10 120 "$R/tools/ubench/valu_rate" > "$OUT/valu_rate.txt" 2>&1
timeout -s KILL 120 rocprofv3 --kernel-trace --stats -d "$OUT/ubtrace" -o trace -- "$R/tools/ubench/valu_rate" \
    > "$OUT/ubtrace.log" 2>&1
timeout -s KILL 120 rocprofv3 --pmc $CNT -d "$OUT/ubpmc" -o pmc -- "$R/tools/ubench/valu_rate" > "$OUT/ubpmc.log" 2>&1
B=(python "$R/bench.py" --steps 5 --warmup 2 --cpu-seconds 0 --no-extras --no-profile)
timeout -s KILL 200 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o trace -- "${B[@]}" > "$OUT/trace.log" 2>&1
timeout -s KILL 200 rocprofv3 --pmc $CNT -d "$OUT/pmc" -o pmc -- "${B[@]}" > "$OUT/pmc.log" 2>&1
python "$R/tools/clock_table.py" "$OUT" > "$OUT/table.txt"
cat "$OUT/valu_rate.txt" "$OUT/table.txt"
