#!/bin/bash
# Round-end evidence on one GPU box, tags prefixed T (default r02f): sort-backend tests, C3 trace +
# FETCH/WRITE, serial C3 trace, blend SQ counters, C4 3/8-strip trace + FETCH/WRITE, every
# single-GPU config bench line, the default bench with the CPU baseline.
set -u
cd "${GRAFT_REPO_ROOT}"
timeout -k 10 300 python -m pytest tests/test_gpu_sort_backend.py -x -q -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/t_sortb.log 2>&1 || { echo "sort tests failed"; tail -5 gpurun_out/t_sortb.log; exit 1; }
tail -1 gpurun_out/t_sortb.log
TAG=${T:-r02f}_c3 bash tools/profile.sh || exit 1
TAG=${T:-r02f}_c3_serial PMC=0 BENCH_ARGS="--steps 30 --warmup 5 --no-cpu-baseline --inflight 1" bash tools/profile.sh || exit 1
TAG=${T:-r02f}_c3 BENCH_ARGS="--steps 10 --warmup 3 --no-cpu-baseline" bash tools/pmc_sq.sh || exit 1
TAG=${T:-r02f}_c4s3 BENCH_ARGS="--config c4 --sim-strip 3/8 --steps 30 --warmup 5 --no-cpu-baseline" bash tools/profile.sh || exit 1
bash tools/configs_bench.sh || exit 1
timeout -k 10 300 python bench.py > gpurun_out/${T:-r02f}_final_bench.log 2>&1 || { echo "bench failed"; exit 1; }
tail -1 gpurun_out/${T:-r02f}_final_bench.log
