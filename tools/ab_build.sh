#!/bin/bash
# Build A/B variants of libfvp.so into ab_libs/<name>.so from the current tree:
#   tools/ab_build.sh name "-DFLAG=1 ..." [name2 "flags2" ...]
set -e
cd "$(dirname "$0")/../faster-voxelpose_amd/csrc"
mkdir -p ../../ab_libs
while [ $# -ge 2 ]; do
  n=$1; f=$2; shift 2
  make -s OBJDIR=build_ab_$n OUT=../../ab_libs/$n.so HIPFLAGS_EXTRA="$f" -j8 >/dev/null
  echo "built ab_libs/$n.so ($f)"
done
