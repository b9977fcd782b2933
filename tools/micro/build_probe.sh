#!/bin/bash
# Builds tools/micro/ds_probe and ds_probe_stop{1,2,3}: the downsweep returns after its loads,
# after sub-pass A, after sub-pass B (see depth_sort.hip GSR_DS_PROBE_STOP).
set -e
cd "$(dirname "$0")"
F="-O3 -std=c++17 -ffp-contract=off -I../../include --offload-arch=gfx950"
/opt/rocm/bin/hipcc $F -o ds_probe ds_probe.hip
for k in 1 2 3; do /opt/rocm/bin/hipcc $F -DGSR_DS_PROBE_STOP=$k -o ds_probe_stop$k ds_probe.hip; done
