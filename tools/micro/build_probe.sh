#!/bin/bash
# Builds tools/micro/ds_probe{,_nostore,_nosubb} (see ds_probe.hip).
set -e
cd "$(dirname "$0")"
F="-O3 -std=c++17 -ffp-contract=off -I../../include --offload-arch=gfx950"
/opt/rocm/bin/hipcc $F -o ds_probe ds_probe.hip
/opt/rocm/bin/hipcc $F -DGSR_DS_PROBE_NO_STORE -o ds_probe_nostore ds_probe.hip
/opt/rocm/bin/hipcc $F -DGSR_DS_PROBE_NO_SUB_B -o ds_probe_nosubb ds_probe.hip
