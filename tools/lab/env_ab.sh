#!/bin/bash
# Interleaved A/B of environment settings (lab switches) on one GPU box, same library: for ROUNDS
# rounds, every ';'-separated env assignment list in ENVS ("-" = none) runs bench.py ARGS.
# Prints: env, frames/s, serial ms per frame, stage times (us).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out/ab
IFS=';' read -ra envs <<< "${ENVS:--}"
for r in $(seq 1 ${ROUNDS:-2}); do
  for e in "${envs[@]}"; do
    [ "$e" = "-" ] && e=""
    env $e timeout -k 10 200 python bench.py --no-cpu-baseline --steps ${STEPS:-200} --warmup 20 ${ARGS:-} > gpurun_out/ab/run.json 2> gpurun_out/ab/run.err || { echo "failed: $e"; tail -5 gpurun_out/ab/run.err; exit 1; }
    python -c "import json; d=json.loads(open('gpurun_out/ab/run.json').read().strip().splitlines()[-1]); print('[$e]', d['value'], d['serial_ms_per_frame'], {k: round(x*1e3,1) for k,x in d['stage_ms'].items()})"
  done
done
