#!/bin/bash
# Interleaved sweep of tuning knobs on one box (C3 by default, BENCH_ARGS to change): each
# entry of KNOBS is "ENV=.. [--bench-flag[=value]]"; "-" is the default.  Prints fps, serial ms and
# stage times per run.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
IFS=';' read -ra knobs <<< "${KNOBS:--}"
for r in $(seq ${ROUNDS:-2}); do
  for k in "${knobs[@]}"; do
    envs=(); flags=()
    for w in $k; do
      case $w in -) ;; --*) flags+=("$w") ;; *) envs+=("$w") ;; esac
    done
    env "${envs[@]}" timeout -k 10 120 python bench.py --steps 200 --warmup 20 --no-cpu-baseline ${BENCH_ARGS:-} "${flags[@]}" > gpurun_out/knob.log 2>&1 || { echo "run [$k] failed"; tail -3 gpurun_out/knob.log; exit 1; }
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['serial_ms_per_frame'], {k: round(x*1e3,1) for k,x in d['stage_ms'].items()})" gpurun_out/knob.log "[$k]"
  done
done
