#!/bin/bash
# tools/profile_config.sh for one config, then its summaries made on the GPU box (the raw
# rocprofv3 output of a 6M-Gaussian run is too large to copy back): gpurun_out/<name>_summary.md,
# profiles-format <name>_kernels.json / <name>_blend_sq.json and the SQ text, raw dir removed.
# Usage: TAG=r03n CONFIG=c4 [EXTRA="--sim-strip 3/8" NAME=c4-strip38] bash tools/profile_summarised.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${TAG:?}; CONFIG=${CONFIG:?}; NAME=${NAME:-$CONFIG}
export TAG CONFIG
TAG=${TAG}_${NAME} bash tools/profile_config.sh || exit 1
D=gpurun_out/prof_${TAG}_${NAME}_${CONFIG}
{ echo "# rocprofv3 summary $TAG $NAME ${EXTRA:-}, serial frames (--inflight 1), lib sha $(cat $D/lib.sha)"
  python tools/prof_summary.py $D --json gpurun_out/${TAG}_${NAME}_kernels.json | sed -n '2,$p'; } \
    > gpurun_out/${TAG}_${NAME}_summary.md || exit 1
python tools/sq_summary.py $D k_blend_q --json gpurun_out/${TAG}_${NAME}_blend_sq.json \
    > gpurun_out/${TAG}_${NAME}_blend_sq.txt || exit 1
rm -rf "$D"
