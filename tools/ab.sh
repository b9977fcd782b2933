#!/bin/bash
# A/B on one box: bench.py with the in-tree library (B) and GSR_LIB=$A_LIB (A), alternated
# ROUNDS times, for each bench argument set in $CASES (separated by ';').
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/ab
A_LIB=${A_LIB:-gaussiansplattingviewer_amd/libgsr_prev.so}
IFS=';' read -ra cases <<< "${CASES:---inflight 1;--inflight 2}"
for r in $(seq 1 ${ROUNDS:-2}); do
  for c in "${cases[@]}"; do
    for v in A B; do
      if [ $v = A ]; then export GSR_LIB=$A_LIB; else unset GSR_LIB; fi
      timeout -k 10 200 python bench.py --no-cpu-baseline --steps 200 --warmup 20 $c > gpurun_out/ab/run.log 2>&1 || { echo "failed: $v $c"; tail -5 gpurun_out/ab/run.log; exit 1; }
      python -c "import json,sys; d=json.loads(open('gpurun_out/ab/run.log').read().strip().splitlines()[-1]); print('$v', '$c', d['value'], {k: round(x*1e3,1) for k,x in d['stage_ms'].items()})"
    done
  done
done
