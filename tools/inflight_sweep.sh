#!/bin/bash
# Frames-in-flight sweep: bench.py at several --inflight depths, HW queue counts and aux
# stream priorities (one JSON line each, summarised at the end).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/inflight
run() {  # tag "VAR=value ..." bench-args...
    local tag=$1 envs=$2; shift 2
    env $envs timeout -k 10 200 python bench.py --no-cpu-baseline --steps 200 --warmup 20 "$@" \
        > gpurun_out/inflight/$tag.log 2>&1 || { echo "$tag failed"; tail -5 gpurun_out/inflight/$tag.log; exit 1; }
}
for spec in ${SPECS:-"d1:GPU_MAX_HW_QUEUES=4:1" "d2:GPU_MAX_HW_QUEUES=4:2" "d2_q8:GPU_MAX_HW_QUEUES=8:2" \
            "d3_q8:GPU_MAX_HW_QUEUES=8:3" "d4_q8:GPU_MAX_HW_QUEUES=8:4" "d2_auxprio0:GSR_AUX_PRIORITY=0:2"}; do
  IFS=: read -r tag envs depth <<< "$spec"
  run "$tag" "$envs" --inflight "$depth" ${ARGS:-} || exit 1
done
for f in gpurun_out/inflight/*.log; do
  python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[1], d['value'], d['roofline']['launch_ms'])" $f
done
