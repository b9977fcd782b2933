#!/bin/bash
# Lab builds (experiments, not the product): libgsr with one csrc/ source replaced by a lab
# variant, as gaussiansplattingviewer_amd/libgsr_lab_<name>.so; bench / tests pick it with
# GSR_LIB=<that path>.  Usage: tools/lab/build.sh <name> <csrc file to replace> <lab source>
set -e
cd "$(dirname "$0")/../.."
name=$1; target=$2; src=$3
make -s -C gaussiansplattingviewer_amd/csrc -j8
OBJ=build/obj; LAB=build/lab_$name; mkdir -p $LAB
F="-O3 -std=c++17 -fPIC -ffp-contract=off -Wall -Wno-unused-function --offload-arch=gfx950 -Iinclude -Igaussiansplattingviewer_amd/csrc"
[ "$target" = blend.hip ] && F="$F -fno-slp-vectorize"
/opt/rocm/bin/hipcc $F ${LAB_FLAGS:-} -c -o $LAB/${target%.hip}.o $src
objs=""
for o in $OBJ/*.o; do b=$(basename $o); if [ "$b" = "${target%.hip}.o" ]; then objs="$objs $LAB/$b"; else objs="$objs $o"; fi; done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o gaussiansplattingviewer_amd/libgsr_lab_$name.so $objs
echo "built gaussiansplattingviewer_amd/libgsr_lab_$name.so"
