#!/bin/bash
# r5t: per-phase instruction / cycle split of k_fast and k_describe after the round-5 cuts
set -uo pipefail
timeout -k 10 900 bash tools/phase_valu.sh measure r05b > gpurun_out/r5t_phase.txt 2>&1; rc=$?; cat gpurun_out/r5t_phase.txt | tail -30; exit $rc
