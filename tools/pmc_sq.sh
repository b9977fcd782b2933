#!/bin/bash
# SQ instruction-mix / stall counters for the bench's kernels (counter passes separate from
# any trace, as MI355X_MICROARCH.md prescribes).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/pmc_${TAG:-sq}
mkdir -p "$OUT"
ARGS=${BENCH_ARGS:---steps 10 --warmup 3 --no-cpu-baseline}
i=0
for set in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" \
           "SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE"; do
  timeout -k 10 600 rocprofv3 --pmc $set --output-format csv -d "$OUT/p$i" -o pmc \
      -- python3 bench.py $ARGS > "$OUT/p$i.log" 2>&1 || { echo "pmc set $i failed"; tail -5 "$OUT/p$i.log"; exit 1; }
  echo "pmc set $i ok"
  i=$((i+1))
done
