#!/bin/bash
# SQ counter calibration run (see valu_calib.hip): two PMC passes over the known kernel.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
OUT=gpurun_out/valu_calib
mkdir -p $OUT
timeout -s KILL 60 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $OUT/p0 -o pmc -- ./tools/micro/valu_calib > $OUT/p0.log 2>&1 || exit 1
timeout -s KILL 60 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_VALU SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE --output-format csv -d $OUT/p1 -o pmc -- ./tools/micro/valu_calib > $OUT/p1.log 2>&1 || echo "p1 failed (counter names?)"
timeout -s KILL 60 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/t -o t -- ./tools/micro/valu_calib > $OUT/t.log 2>&1 || exit 1
echo done
