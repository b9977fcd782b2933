#!/bin/bash
# GPU-box evidence run, tag T (default r03): smoke -> the GPU parity suite -> blend error vs the
# oracle at C2-C5 in both arithmetic modes.  Every GPU step has its own time limit; anything but
# a plain test failure ends the script.  Outputs under gpurun_out/ (copy what is judged to profiles/).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
T=${T:-r03}
mkdir -p gpurun_out
step() {  # name seconds cmd...
    local name=$1 secs=$2
    shift 2
    local t0=$(date +%s)
    timeout -k 10 "$secs" "$@" > "gpurun_out/${T}_$name.txt" 2>&1
    local rc=$?
    echo "[$name] rc=$rc ($(( $(date +%s) - t0 )) s)"
    tail -n 3 "gpurun_out/${T}_$name.txt"
    return $rc
}
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" || exit 1
if [ "${SKIP_TESTS:-0}" != "1" ]; then
    step gpu_tests "${TEST_SECS:-900}" python -u -m pytest tests -m gpu -x -v -p no:cacheprovider \
        --timeout 300 --timeout-method thread ${PYTEST_ARGS:-}
    rc=$?
    if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit 1; fi
fi
if [ "${ERR_STATS:-1}" = "1" ]; then
    step blend_error 600 python -u tools/blend_error_stats.py --configs ${ERR_CONFIGS:-c2,c3,c4,c5} || exit 1
fi
