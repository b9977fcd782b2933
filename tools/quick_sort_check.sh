#!/bin/bash
# Depth-sort iteration on the GPU box: sort-backend + parity tests, then a serial rocprofv3
# kernel trace of the C3 bench and the bench line.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider ${TESTS:-tests/test_gpu_sort_backend.py tests/test_gpu_parity.py} > gpurun_out/qs_tests.log 2>&1
rc=$?; tail -4 gpurun_out/qs_tests.log; [ $rc -le 1 ] || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_${TAG:-qs}/trace -o trace -- python3 bench.py --steps 30 --warmup 5 --no-cpu-baseline --inflight 1 ${BENCH_ARGS:-} > gpurun_out/qs_prof.log 2>&1 || { echo "prof rc=$?"; exit 1; }
timeout -k 10 300 python bench.py --steps 100 --warmup 10 --no-cpu-baseline ${BENCH_ARGS:-} > gpurun_out/qs_bench.log 2>&1 || { echo "bench rc=$?"; exit 1; }
python3 -c "import json; d=json.loads(open('gpurun_out/qs_bench.log').read().strip().splitlines()[-1]); print(d['value'], d['serial_ms_per_frame'], d['stage_ms'])"
