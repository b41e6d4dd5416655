#!/bin/bash
# r6e: round-6 state after the f16 arc network: GPU suite, VGA / FHD / FHD-stereo
# profiles, the bench line; then the k_fast / k_describe phase split
set -uo pipefail
bash tools/round_measure.sh r06b || exit 1
timeout -k 10 600 bash tools/phase_valu.sh measure r06b > gpurun_out/phase_valu_r06b.txt 2>&1 || { tail -20 gpurun_out/phase_valu_r06b.txt; exit 1; }
tail -20 gpurun_out/phase_valu_r06b.txt
