#!/bin/bash
# r6q: fast local BA -- k_ba_chol_fast (pipelined panel, blocked back solve) clocks, fused Schur pairs, A/B
set -uo pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_ba.py > gpurun_out/r6q_pytest.txt 2>&1 || { tail -40 gpurun_out/r6q_pytest.txt; exit 1; }
tail -1 gpurun_out/r6q_pytest.txt
ORBX_BA_CLOCKS=1 timeout -k 10 120 python tools/ba_fast_probe.py 5 2>&1 | grep -v amdgpu.ids
: > gpurun_out/r6q_ab_ba.txt
for r in 1 2 3; do
  for E in X=0 ORBX_BA_CHOL_FAST=0 ORBX_BA_PAIRS_FUSED=0; do
    echo "$E $(env $E timeout -k 10 120 python tools/ba_fast_probe.py 5 2>/dev/null | tr '\n' ' ')" >> gpurun_out/r6q_ab_ba.txt || exit 1
  done
done
cat gpurun_out/r6q_ab_ba.txt
