#!/bin/bash
# Builds liborbx from a git revision's kernel sources into
# orb_slam_2_ros_amd/liborbx_<name>.so, for same-box A/B timing with
# tools/ab_bench.sh (ORBX_LIB selects the library).
#   tools/build_variant.sh REV NAME [extra hipcc flags]     (REV = WORKTREE: the working tree)
set -euo pipefail
REV=$1; NAME=$2; shift 2
R=$(cd "$(dirname "$0")/.." && pwd)
T=$(mktemp -d /tmp/orbx_var.XXXX)
mkdir -p "$T/pkg/csrc" "$T/include"
if [ "$REV" = WORKTREE ]; then   # the working tree's sources (with other -D flags)
    cp "$R"/orb_slam_2_ros_amd/csrc/*.hip "$R"/orb_slam_2_ros_amd/csrc/*.h "$R"/orb_slam_2_ros_amd/csrc/*.inc \
       "$R"/orb_slam_2_ros_amd/csrc/Makefile "$T/pkg/csrc/"
    cp "$R/include/orbx.h" "$T/include/orbx.h"
else
    for f in $(git -C "$R" ls-tree --name-only "$REV" orb_slam_2_ros_amd/csrc/); do
        git -C "$R" show "$REV:$f" > "$T/pkg/csrc/$(basename "$f")"
    done
    git -C "$R" show "$REV:include/orbx.h" > "$T/include/orbx.h"
fi
make -s -j8 -C "$T/pkg/csrc" ${1:+CXXFLAGS="$*"} > /dev/null
cp "$T/pkg/liborbx.so" "$R/orb_slam_2_ros_amd/liborbx_$NAME.so"
rm -rf "$T"
echo "built orb_slam_2_ros_amd/liborbx_$NAME.so from $REV"
