#!/bin/bash
# GPU-box session: smoke -> GPU parity tests -> bench.  Each GPU step runs under its own
# time limit; a crash, abort or timeout (anything but a plain test failure) ends the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
run() {  # name seconds cmd...
    local name=$1 secs=$2
    shift 2
    local t0=$(date +%s)
    timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
    local rc=$?
    echo "[$name] rc=$rc ($(( $(date +%s) - t0 )) s)"
    tail -n 5 "gpurun_out/$name.log"
    return $rc
}
run smoke 400 python -c "import __graft_entry__ as g; g.smoke()" || exit 1
if [ "${SKIP_TESTS:-0}" != "1" ]; then
    run pytest_gpu "${TEST_SECS:-900}" python -m pytest tests -m gpu -q -p no:cacheprovider ${PYTEST_ARGS:-}
    rc=$?
    if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit 1; fi
fi
run bench 600 python bench.py ${BENCH_ARGS:---steps 100 --warmup 10} || exit 1
