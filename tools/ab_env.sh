#!/bin/bash
# Interleaved A/B of environment settings on one box: `tools/ab_env.sh "ENV_A" "ENV_B" [reps]`
# runs the C3 bench alternately under each setting (e.g. "GSR_COLOR_BLOCKS=512") and prints the
# frame rate, serial frame time and stage times of every run.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
A=$1; B=$2; N=${3:-3}
for i in $(seq $N); do
  for v in A B; do
    E=${!v}
    env $E timeout -k 10 120 python bench.py --steps 200 --warmup 20 --no-cpu-baseline ${BENCH_ARGS:-} > gpurun_out/ab_$v.log 2>&1 || { echo "run $v failed"; tail -3 gpurun_out/ab_$v.log; exit 1; }
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['serial_ms_per_frame'], {k: round(x*1e3,1) for k,x in d['stage_ms'].items()})" gpurun_out/ab_$v.log "$v[$E]"
  done
done
