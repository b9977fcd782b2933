#!/bin/bash
# Serial kernel traces of several library builds for one bench case (lab): for every name in
# LIBS ("base" = the in-tree libgsr.so, X = libgsr_lab_X.so), rocprofv3 --kernel-trace --stats of
# `bench.py $ARGS --inflight 1` into gpurun_out/trace_ab/<name>/.  Summarise with
#   python tools/prof_summary.py gpurun_out/trace_ab/<name>
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
for v in ${LIBS:-base}; do
  if [ "$v" = base ]; then unset GSR_LIB; else export GSR_LIB=$PWD/gaussiansplattingviewer_amd/libgsr_lab_$v.so; fi
  mkdir -p gpurun_out/trace_ab/$v
  timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/trace_ab/$v/trace -o trace \
    -- python3 bench.py ${ARGS:---config c3} --inflight 1 --steps 30 --warmup 5 --no-cpu-baseline \
    > gpurun_out/trace_ab/$v/trace.log 2>&1 || { echo "$v failed"; tail -5 gpurun_out/trace_ab/$v/trace.log; exit 1; }
  echo "$v ok"
done
