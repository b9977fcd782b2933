#!/bin/bash
# Sweep one environment knob on one box: `VAR=GSR_COLOR_WAVES VALUES="0 2 4" tools/env_sweep.sh`
# runs the bench (BENCH_ARGS, default C3) once per value per round (ROUNDS, default 2), values
# interleaved, and prints the frame rate, serial frame time and stage times of every run.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for r in $(seq ${ROUNDS:-2}); do
  for v in $VALUES; do
    env $VAR=$v timeout -k 10 150 python bench.py --steps 200 --warmup 20 --no-cpu-baseline ${BENCH_ARGS:-} > gpurun_out/sweep.log 2>&1 || { echo "run $v failed"; tail -3 gpurun_out/sweep.log; exit 1; }
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['serial_ms_per_frame'], {k: round(x*1e3,1) for k,x in d['stage_ms'].items()})" gpurun_out/sweep.log "$VAR=$v ${BENCH_ARGS:-}"
  done
done
