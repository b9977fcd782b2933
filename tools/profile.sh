#!/bin/bash
# rocprofv3 kernel trace + stats of the bench, then HBM counters (FETCH_SIZE and WRITE_SIZE
# in separate passes, as MI355X_MICROARCH.md's rocprofv3 section prescribes).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/prof_${TAG:-run}
mkdir -p "$OUT"
ARGS=${BENCH_ARGS:---steps 30 --warmup 5 --no-cpu-baseline}
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o trace \
    -- python3 bench.py $ARGS > "$OUT/trace.log" 2>&1 || { echo "trace failed rc=$?"; tail -20 "$OUT/trace.log"; exit 1; }
echo "trace ok"; tail -1 "$OUT/trace.log"
if [ "${PMC:-1}" = "1" ]; then
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -k 10 600 rocprofv3 --pmc $c --output-format csv -d "$OUT/pmc_$c" -o pmc \
        -- python3 bench.py $ARGS > "$OUT/pmc_$c.log" 2>&1 || { echo "pmc $c failed rc=$?"; tail -20 "$OUT/pmc_$c.log"; exit 1; }
    echo "pmc $c ok"
  done
fi
find "$OUT" -name "*.csv" | head -20
