#!/bin/bash
# rocprofv3 evidence for one bench config on the GPU box, serial frames (--inflight 1, so each
# kernel's duration is its own): a kernel trace + stats, then HBM counters (FETCH_SIZE and
# WRITE_SIZE in separate passes, as MI355X_MICROARCH.md's rocprofv3 section prescribes), then
# two SQ counter sets for the blend.  Each pass runs under its own time limit; the first failure
# ends the script.  Writes gpurun_out/prof_${TAG}_${CONFIG}/ and the sha of the profiled
# library (lib.sha); summarise here with
#   python tools/prof_summary.py gpurun_out/prof_<tag>_<config> --json profiles/<tag>_<config>_kernels.json
#   python tools/sq_summary.py gpurun_out/prof_<tag>_<config> k_blend_q --json profiles/<tag>_<config>_blend_sq.json
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
CONFIG=${CONFIG:-c3}
TAG=${TAG:-r03}
OUT=gpurun_out/prof_${TAG}_${CONFIG}
mkdir -p "$OUT"
sha256sum gaussiansplattingviewer_amd/libgsr.so | cut -c1-16 > "$OUT/lib.sha"
ARGS="--config $CONFIG --inflight 1 --steps ${STEPS:-30} --warmup 5 --no-cpu-baseline ${EXTRA:-}"
pass() {  # name rocprof-args...
    local name=$1; shift
    timeout -k 10 ${PASS_SECS:-300} rocprofv3 "$@" --output-format csv -d "$OUT/$name" -o pmc \
        -- python3 bench.py $ARGS > "$OUT/$name.log" 2>&1 || { echo "$CONFIG $name failed rc=$?"; tail -5 "$OUT/$name.log"; exit 1; }
    echo "$CONFIG $name ok"
}
timeout -k 10 ${PASS_SECS:-300} rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o trace \
    -- python3 bench.py $ARGS > "$OUT/trace.log" 2>&1 || { echo "$CONFIG trace failed rc=$?"; tail -5 "$OUT/trace.log"; exit 1; }
echo "$CONFIG trace ok: $(tail -c 300 "$OUT/trace.log" | tr '\n' ' ')"
if [ "${PMC:-1}" = "1" ]; then
    pass pmc_FETCH_SIZE --pmc FETCH_SIZE
    pass pmc_WRITE_SIZE --pmc WRITE_SIZE
fi
if [ "${SQ:-1}" = "1" ]; then
    pass p0 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE
    pass p1 --pmc SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE
fi
