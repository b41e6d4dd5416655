#!/bin/bash
# Per-phase instruction split of k_fast and k_describe.
#   tools/phase_valu.sh build        (CPU) the stop-after-phase-N builds, from the working tree:
#                                    orb_slam_2_ros_amd/liborbx_stopf{1..4}.so, liborbx_stopd{1,2,4}.so
#   tools/phase_valu.sh measure TAG  (GPU) one rocprofv3 --pmc pass per build and the product,
#                                    VGA bench workload; prints the split (tools/phase_valu.py)
set -uo pipefail
R=$(cd "$(dirname "$0")/.." && pwd)
CTRS="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_MFMA SQ_INSTS_VMEM SQ_WAVE_CYCLES"
case "$1" in
build)
    T=$(mktemp -d /tmp/orbx_stop.XXXX)
    for v in f1 f2 f3 f4 d1 d2 d4; do
        mkdir -p "$T/$v/pkg/csrc" "$T/$v/include"
        cp "$R"/orb_slam_2_ros_amd/csrc/*.hip "$R"/orb_slam_2_ros_amd/csrc/*.h "$R"/orb_slam_2_ros_amd/csrc/*.inc \
           "$R"/orb_slam_2_ros_amd/csrc/Makefile "$T/$v/pkg/csrc/"
        cp "$R/include/orbx.h" "$T/$v/include/"
        def=$([ "${v:0:1}" = f ] && echo "-DORBX_STOP_FAST=${v:1}" || echo "-DORBX_STOP_DESC=${v:1}")
        (make -s -j4 -C "$T/$v/pkg/csrc" \
            CXXFLAGS="-O3 -std=c++17 -fPIC -ffp-contract=off -fno-slp-vectorize -Wall -Wno-unused-function $def" \
            > /dev/null && cp "$T/$v/pkg/liborbx.so" "$R/orb_slam_2_ros_amd/liborbx_stop$v.so") &
    done
    wait
    rm -rf "$T"
    ls "$R"/orb_slam_2_ros_amd/liborbx_stop*.so
    ;;
measure)
    TAG=$2
    OUT=$R/gpurun_out/phase_valu_$TAG
    mkdir -p "$OUT"
    cd /tmp && export TMPDIR=/tmp ORBX_SPLIT=1 ORBX_PIPELINE=0
    for v in full f1 f2 f3 f4 d1 d2 d4; do
        lib=$R/orb_slam_2_ros_amd/liborbx.so
        [ "$v" != full ] && lib=$R/orb_slam_2_ros_amd/liborbx_stop$v.so
        echo "pass $v"
        ORBX_LIB=$lib timeout -s KILL 200 rocprofv3 --pmc $CTRS -d "$OUT/$v" -o pmc -- python "$R/bench.py" \
            --steps 2 --warmup 1 --cpu-seconds 0 --no-extras --no-profile > "$OUT/$v.log" 2>&1 \
            || { echo "pass $v failed"; tail -3 "$OUT/$v.log"; exit 1; }
    done
    cd "$R" && python tools/phase_valu.py "$OUT"
    ;;
esac
