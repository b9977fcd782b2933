#!/bin/bash
# Lab builds of the whole library with extra compile flags (experiment-only -D switches of a lab source):
# gaussiansplattingviewer_amd/libgsr_lab_<name>.so; bench / tests pick it with GSR_LIB=<path>.
# Usage: tools/lab/build_all.sh <name> <flags...>
set -e
cd "$(dirname "$0")/../.."
name=$1; shift
LAB=build/lab_all_$name; mkdir -p $LAB
F="-O3 -std=c++17 -fPIC -ffp-contract=off -Wall -Wno-unused-function --offload-arch=gfx950 -Iinclude -Igaussiansplattingviewer_amd/csrc $*"
objs=""
for src in api preprocess depth_sort radix_sort binning blend ply_loader stereo; do
  extra=""; [ $src = blend ] || [ $src = preprocess ] && extra="-fno-slp-vectorize"
  /opt/rocm/bin/hipcc $F $extra -c -o $LAB/$src.o gaussiansplattingviewer_amd/csrc/$src.hip &
  objs="$objs $LAB/$src.o"
done
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o gaussiansplattingviewer_amd/libgsr_lab_$name.so $objs
echo "built gaussiansplattingviewer_amd/libgsr_lab_$name.so"
