#!/bin/bash
# Driver-shaped bench runs on one fresh box: the driver's own command (`bench.py --gpus 1 --steps
# 20 --warmup 5`, CPU baseline included) first, as the box's first GPU process, then again, then
# interleaved variants (VARIANTS: ';'-separated extra bench arguments, "-" = none).  Prints one
# line per run: order, variant, frames/s, ms per step, serial ms, in-flight blend ms, inflight.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/ds
IFS=';' read -ra vars <<< "${VARIANTS:--;--inflight 2}"
n=0
one() {  # variant args...
    local v=$1; shift
    n=$((n + 1))
    timeout -k 10 240 python3 bench.py --gpus 1 --steps ${STEPS:-20} --warmup ${WARMUP:-5} "$@" \
        > gpurun_out/ds/run$n.json 2> gpurun_out/ds/run$n.err || { echo "failed: $v"; tail -5 gpurun_out/ds/run$n.err; exit 1; }
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline']; print(sys.argv[2], repr(sys.argv[3]), d['value'], d['ms_per_step'], d['serial_ms_per_frame'], r['launch_ms'], r['launch_ms_inflight'], d['inflight'], d.get('streams'))" gpurun_out/ds/run$n.json $n "$v"
}
one driver
one driver --no-cpu-baseline
for r in $(seq 1 ${ROUNDS:-2}); do
  for v in "${vars[@]}"; do
    if [ "$v" = "-" ]; then one "-" --no-cpu-baseline; else one "$v" --no-cpu-baseline $v; fi
  done
done
