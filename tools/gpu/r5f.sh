#!/bin/bash
set -uo pipefail
mkdir -p gpurun_out
bash tools/gpu/r5d.sh > /dev/null 2>&1 || { tail -5 gpurun_out/r5d_call_ab.txt; exit 1; }
cat gpurun_out/r5d_call_ab.txt
for x in host_fed_vga host_fed_fhd; do
  timeout -k 10 300 python bench.py --extra $x --steps 20 --warmup 3 > gpurun_out/r5f_$x.log 2>&1 || { tail -5 gpurun_out/r5f_$x.log; exit 1; }
  tail -1 gpurun_out/r5f_$x.log
done
