#!/bin/bash
# Quick check on the GPU box: parity + config tests, C4 strip 3/8 and C3 bench lines, a serial
# C3 rocprofv3 kernel trace (gpurun_out/prof_${TAG}_serial).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider ${TESTS:-tests/test_gpu_parity.py tests/test_gpu_configs.py} > gpurun_out/cc_tests.log 2>&1
rc=$?; tail -2 gpurun_out/cc_tests.log; [ $rc -le 1 ] || exit 1
for c in "--config c4 --sim-strip 3/8 --steps 100 --warmup 10" "--config c3 --steps 200 --warmup 20"; do
  timeout -k 10 200 python bench.py --no-cpu-baseline $c > gpurun_out/cc_b.log 2>&1 || { echo "bench failed: $c"; tail -3 gpurun_out/cc_b.log; exit 1; }
  python3 -c "import json,sys; d=json.loads(open('gpurun_out/cc_b.log').read().strip().splitlines()[-1]); print(sys.argv[1], d['value'], d['serial_ms_per_frame'], {k: round(x*1e3,1) for k,x in d['stage_ms'].items()})" "$c"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_${TAG:-cc}_serial/trace -o trace -- python3 bench.py --steps 30 --warmup 5 --no-cpu-baseline --inflight 1 > gpurun_out/cc_prof.log 2>&1 || { echo "prof failed"; exit 1; }
echo ok
