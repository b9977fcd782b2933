#!/bin/bash
# The round's whole evidence for the in-tree library, tag T, in one GPU call: tools/final_evidence.sh
# (smoke, the GPU suite, the serial C3 profile, the default bench line), tools/final_configs.sh
# (every other config's profile and bench line), then driver-shaped runs of the headline.
# Summaries land under gpurun_out/ (copy them to profiles/).  The first failure ends it.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
T=${T:?set T}
export T TMPDIR=/tmp
bash tools/final_evidence.sh > gpurun_out/${T}_evidence.log 2>&1 || { tail -30 gpurun_out/${T}_evidence.log; exit 1; }
tail -4 gpurun_out/${T}_evidence.log
bash tools/final_configs.sh > gpurun_out/${T}_final_configs.log 2>&1 || { tail -30 gpurun_out/${T}_final_configs.log; exit 1; }
cat gpurun_out/${T}_configs_bench.txt
VARIANTS="-" ROUNDS=1 bash tools/driver_shape.sh > gpurun_out/${T}_driver_shape.txt 2>&1 || exit 1
cut -d' ' -f1-8 gpurun_out/${T}_driver_shape.txt
