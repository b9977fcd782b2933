#!/bin/bash
# Round-end evidence on one GPU box (each step under its own time limit; stops at the first
# failure): C3 rocprofv3 trace + FETCH/WRITE passes, blend SQ counters, a C4 1/8-strip trace +
# PMC, every single-GPU config's bench line, the default bench with the CPU baseline.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
T=${TAG:-r02}
TAG=${T}_c3 bash tools/profile.sh || exit 1
TAG=${T}_c3 BENCH_ARGS="--steps 10 --warmup 3 --no-cpu-baseline" bash tools/pmc_sq.sh || exit 1
TAG=${T}_c4s3 BENCH_ARGS="--config c4 --sim-strip 3/8 --steps 30 --warmup 5 --no-cpu-baseline" bash tools/profile.sh || exit 1
bash tools/configs_bench.sh || exit 1
timeout -k 10 300 python bench.py > gpurun_out/${T}_final_bench.log 2>&1 || { echo "bench failed"; exit 1; }
tail -1 gpurun_out/${T}_final_bench.log
