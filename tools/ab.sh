#!/bin/bash
# Interleaved A/B of library builds on one GPU box: for ROUNDS rounds, every bench argument set
# in CASES (';'-separated) with every library in LIBS (space-separated names: "base" = the
# in-tree libgsr.so, X = gaussiansplattingviewer_amd/libgsr_lab_X.so, tools/lab/build.sh).
# Prints one line per run: library, case, frames/s, serial ms per frame, stage times (us).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/ab
IFS=';' read -ra cases <<< "${CASES:---inflight 1;--inflight 2}"
for r in $(seq 1 ${ROUNDS:-2}); do
  for c in "${cases[@]}"; do
    for v in ${LIBS:-base}; do
      if [ "$v" = base ]; then unset GSR_LIB; else export GSR_LIB=$PWD/gaussiansplattingviewer_amd/libgsr_lab_$v.so; fi
      timeout -k 10 200 python bench.py --no-cpu-baseline --steps ${STEPS:-200} --warmup 20 $c > gpurun_out/ab/run.json 2> gpurun_out/ab/run.err || { echo "failed: $v $c"; tail -5 gpurun_out/ab/run.err; exit 1; }
      python -c "import json; d=json.loads(open('gpurun_out/ab/run.json').read().strip().splitlines()[-1]); print('$v', '$c', d['value'], d['serial_ms_per_frame'], {k: round(x*1e3,1) for k,x in d['stage_ms'].items()})"
    done
  done
done
unset GSR_LIB
